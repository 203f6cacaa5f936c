"""Dev A/B (GPU box): top-k variant libraries built by tools/ab/build.sh, timed on the
configs[3] factors after two iterations (sample of users x all 1M items), plus an
agreement check of every variant against v0.
    python tools/ab/topk_ab.py [sample_users] [variants...]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import _pkgload  # noqa: E402

_pkgload.load()
from als_mi355x import datasets as D, engine as E  # noqa: E402


def main():
    ml = len(sys.argv) > 1 and sys.argv[1] == "ml25m"  # configs[1] shape, rank 64, all users
    s = 0 if ml else (int(sys.argv[1]) if len(sys.argv) > 1 else 262144)
    variants = sys.argv[2:] or open(os.path.join(ROOT, "tools", "ab", "variants.txt")).read().split()
    dev = torch.device("cuda", 0)
    k = 64 if ml else 128
    u, i, r = D.synthetic_config("ml25m", device=dev) if ml else D.big_config("big1b", device=dev)
    core = E.ALSCore(u, i, r, device=dev)
    del u, i, r
    torch.cuda.empty_cache()
    core.init_factors(k, seed=5)
    for _ in range(2):
        core.iterate(0.1)
    torch.cuda.synchronize()
    s = s or core.n_users
    Q = core.U[:s].contiguous()
    V = core.V
    n_v = core.n_items
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    ref = {}
    for v in variants:
        L = ctypes.CDLL(os.path.join(ROOT, "tools", "ab", f"libtk_{v}.so"))
        L.ab_topk.argtypes = [P, I64, P, I64, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P,
                              ctypes.c_size_t, P]
        L.ab_ws.argtypes = [I64, I64, ctypes.c_int, ctypes.c_int]
        L.ab_ws.restype = ctypes.c_size_t
        for top in (10, 100):
            ws = torch.empty(int(L.ab_ws(s, n_v, k, top)) + 4096, dtype=torch.uint8, device=dev)
            idx = torch.empty((s, top), dtype=torch.int32, device=dev)
            sc = torch.empty((s, top), dtype=torch.float32, device=dev)
            st = torch.cuda.current_stream().cuda_stream
            args = (Q.data_ptr(), s, V.data_ptr(), n_v, Q.shape[1], k, top, idx.data_ptr(),
                    sc.data_ptr(), ws.data_ptr(), ws.numel(), st)
            assert L.ab_topk(*args) == 0
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert L.ab_topk(*args) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            key = top
            if key not in ref:
                ref[key] = (idx.clone(), sc.clone())
            agree = float((idx == ref[key][0]).float().mean())
            dsc = float((sc - ref[key][1]).abs().max())
            print(f"{v} top{top}: {min(ts):.1f} ms (runs {[round(t, 1) for t in ts]}) "
                  f"agree_vs_first {agree:.5f} max|dscore| {dsc:.2e}", flush=True)


if __name__ == "__main__":
    main()
