"""Dev: configs[4] top-10 / top-100 timing on configs[3]-shaped factors (2 ALS
iterations from the seed), for the library ALS_HIP_LIB points at.
    python tools/topk_big.py [sample]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import _pkgload  # noqa: E402

_pkgload.load()
from als_mi355x import datasets as D, engine as E  # noqa: E402


def main():
    s = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    dev = torch.device("cuda", 0)
    u, i, r = D.big_config("big1b", device=dev)
    core = E.ALSCore(u, i, r, device=dev)
    del u, i, r
    torch.cuda.empty_cache()
    core.init_factors(128, seed=5)
    for _ in range(2):
        core.iterate(0.1)
    torch.cuda.synchronize()
    Q = core.U[:s].contiguous()
    lib = os.environ.get("ALS_HIP_LIB", "default")
    if "--count" in sys.argv:  # offers per wave (tools/libals_topk_dev.so, MODE 3)
        import ctypes
        from als_mi355x import _lib
        L = ctypes.CDLL(os.path.join(ROOT, "tools", "libals_topk_dev.so"))
        P, I64 = ctypes.c_void_p, ctypes.c_int64
        L.dev_topk.argtypes = [ctypes.c_int, P, I64, P, I64, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, P, P, P, ctypes.c_size_t, P, P]
        n_v = core.n_items
        for top in (10, 100):
            ws = torch.empty(int(_lib.lib().als_topk_workspace_bytes(s, n_v, 128, top)),
                             dtype=torch.uint8, device=dev)
            idx = torch.empty((s, top), dtype=torch.int32, device=dev)
            sc = torch.empty((s, top), dtype=torch.float32, device=dev)
            dbg = torch.zeros(s * 4 + 64, dtype=torch.float32, device=dev)
            st = torch.cuda.current_stream().cuda_stream
            for mode in (0, 3):
                rc = L.dev_topk(mode, Q.data_ptr(), s, core.V.data_ptr(), n_v, Q.shape[1], 128, top,
                                idx.data_ptr(), sc.data_ptr(), ws.data_ptr(), ws.numel(),
                                dbg.data_ptr(), st)
                assert rc == 0, rc
            torch.cuda.synchronize()
            rg = 2 if top <= 16 else 1
            waves = (s + 64 * rg - 1) // (64 * rg) * 4
            cnt = dbg[:waves].double()
            blocks = (n_v + 15) // 16 * rg
            print(f"top{top}: offers/wave mean {float(cnt.mean()):.0f} max {float(cnt.max()):.0f} "
                  f"of {blocks} blocks", flush=True)
    for top in (10, 100):
        E.topk_rows(Q, s, core.V, core.n_items, 128, top)
        torch.cuda.synchronize()
        ts = []
        for _ in range(2):
            t0 = time.perf_counter()
            E.topk_rows(Q, s, core.V, core.n_items, 128, top)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"{lib} top{top}: {1e3 * min(ts):.1f} ms  {s / min(ts) / 1e6:.3f} M recs/s", flush=True)


if __name__ == "__main__":
    main()
