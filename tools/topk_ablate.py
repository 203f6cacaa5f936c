"""Dev tool (GPU box): time topk_split_kernel ablation modes on bench-shaped factors.
    python tools/topk_ablate.py --build      (here, cross-compiles tools/libals_topk_dev.so)
    python tools/topk_ablate.py [--rank K] [--top T]
Factors: one ALS iteration on the ML-25M-shaped synthetic data (as bench.py)."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "tools", "libals_topk_dev.so")


def build():
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950",
                           "-std=c++17", os.path.join(ROOT, "tools", "dev_topk.hip"), "-o", SO])


def main():
    if "--build" in sys.argv:
        build()
        return
    import torch
    import _pkgload
    _pkgload.load()
    from als_mi355x import datasets as D, engine as E
    a = sys.argv
    k = int(a[a.index("--rank") + 1]) if "--rank" in a else 64
    top = int(a[a.index("--top") + 1]) if "--top" in a else 10
    L = ctypes.CDLL(SO)
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    L.dev_topk.argtypes = [ctypes.c_int, P, I64, P, I64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           P, P, P, ctypes.c_size_t, P, P]
    dev = torch.device("cuda", 0)
    u, i, r = D.synthetic_config("ml25m", device=dev)
    core = E.ALSCore(u, i, r, device=dev)
    core.init_factors(k, seed=5)
    core.iterate(0.1)
    torch.cuda.synchronize()
    Q, V, n_q, n_v = core.U, core.V, core.n_users, core.n_items
    from als_mi355x import _lib
    ws = torch.empty(int(_lib.lib().als_topk_workspace_bytes(n_q, n_v, k, top)),
                     dtype=torch.uint8, device=dev)
    idx = torch.empty((n_q, top), dtype=torch.int32, device=dev)
    sc = torch.empty((n_q, top), dtype=torch.float32, device=dev)
    dbg = torch.zeros(n_q * 4 + 64, dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def run(mode):
        rc = L.dev_topk(mode, Q.data_ptr(), n_q, V.data_ptr(), n_v, Q.shape[1], k, top,
                        idx.data_ptr(), sc.data_ptr(), ws.data_ptr(), ws.numel(), dbg.data_ptr(), st)
        assert rc == 0, rc

    run(0)
    torch.cuda.synchronize()
    for mode in (0, 1, 2, 3, 0):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(mode)
        e1.record()
        torch.cuda.synchronize()
        extra = ""
        if mode == 3:
            waves = (n_q + 127) // 128 * 4
            cnt = dbg[:waves].double()
            blocks = (n_v + 15) // 16 * 2
            extra = (f" offers/wave mean {float(cnt.mean()):.0f} max {float(cnt.max()):.0f} "
                     f"of {blocks} blocks ({100 * float(cnt.mean()) / blocks:.1f}%)")
        print(f"rank {k} top {top} mode {mode}: {e0.elapsed_time(e1):.3f} ms{extra}", flush=True)


if __name__ == "__main__":
    main()
