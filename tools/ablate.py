"""Dev tool: time the phases of the explicit light-row half-sweep kernels on the
ML-25M-shaped synthetic data (tools/dev_ablate.hip: full / Gram only / solve only).
    python tools/ablate.py --build          (CPU: hipcc -> tools/libals_dev.so)
    python tools/ablate.py [--rank 64|128] [--config big1b]  (GPU box; big1b: configs[3], items only)
Prints ms per launch and ns per row for each mode on the item and the user side."""
import ctypes
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import _pkgload  # noqa: E402

_pkgload.load()
from als_mi355x import datasets as D, engine as E  # noqa: E402

SO = os.path.join(ROOT, "tools", "libals_dev.so")
if "--lib" in sys.argv:  # a tools/ab/variant.py --dev build
    SO = sys.argv[sys.argv.index("--lib") + 1]


def build():
    src = os.path.join(ROOT, "tools", "dev_ablate.hip")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950",
                           "-std=c++17", src, "-o", SO])


def split_table(Y, k, kp):
    """The explicit path's split table (as split_table_kernel): hi | lo << 16 of 2^ey * Y,
    kp words per row, plus the zero row."""
    ey = 14 - math.floor(math.log2(float(Y[:, :k].abs().max())))
    t = Y[:, :k].float() * (2.0 ** ey)
    hi = t.half()
    lo = (t - hi.float()).half()
    w = (hi.view(torch.int16).to(torch.int32) & 0xFFFF) | (lo.view(torch.int16).to(torch.int32) << 16)
    out = torch.zeros((Y.shape[0] + 1, kp), dtype=torch.int32, device=Y.device)
    out[:-1, :k] = w
    return out.contiguous(), ey


def main():
    if "--build" in sys.argv:
        build()
        return
    k = int(sys.argv[sys.argv.index("--rank") + 1]) if "--rank" in sys.argv else 64
    nb = 4 if k <= 64 else 8
    kp = 16 * nb
    L = ctypes.CDLL(SO)
    P, F, I = ctypes.c_void_p, ctypes.c_float, ctypes.c_int
    L.dev_ablate.argtypes = [I, I, P, P, P, P, I, P, I, I, F, F, F, P, I, I, F, P, P, P]
    dev = torch.device("cuda", 0)
    big = "--config" in sys.argv and sys.argv[sys.argv.index("--config") + 1] == "big1b"
    u, i, r = D.big_config("big1b", device=dev) if big else D.synthetic_config("ml25m", device=dev)
    core = E.ALSCore(u, i, r, device=dev)
    del u, i, r
    torch.cuda.empty_cache()
    core.init_factors(k, seed=5)
    core.iterate(0.1)
    torch.cuda.synchronize()
    rcnt = torch.zeros(2, dtype=torch.int32, device=dev)
    names = {0: "full", 1: "gram only", 2: "solve only"}
    sides = (("item", core.item_block, core.U, core.V),
             ("user", core.user_block, core.V, core.U))
    for side, blk, Y, X in sides[:1] if big else sides:
        n = blk.n_light - blk.n_dual(k)  # the primal light rows (the dual tail has its own kernel)
        lr = blk.light_rows[:n].long()
        lnnz = int((blk.row_ptr[lr + 1] - blk.row_ptr[lr]).sum())
        print(f"{side}: light {blk.n_light} (primal {n}, {lnnz} ratings), heavy {blk.n_heavy}, "
              f"chunks {blk.n_chunks}, nnz {int(blk.row_ptr[-1])}", flush=True)
        X2 = torch.empty_like(X)
        rlist = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
        Ysp, ey = split_table(Y, k, kp)
        er = 14 - math.floor(math.log2(float(blk.val.abs().max())))
        for mode in (0, 1, 2):
            times = []
            for rep in range(4):
                rcnt.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = L.dev_ablate(nb, mode, blk.row_ptr.data_ptr(), blk.col.data_ptr(),
                                  blk.val.data_ptr(), blk.light_rows.data_ptr(), n, Ysp.data_ptr(),
                                  kp, Y.shape[0], 2.0 ** er, 2.0 ** (-2 * ey), 2.0 ** (-ey - er),
                                  X2.data_ptr(), X.shape[1], k, 0.1, rcnt.data_ptr(),
                                  rlist.data_ptr(), torch.cuda.current_stream().cuda_stream)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, rc
                times.append(e0.elapsed_time(e1))
            t = sorted(times[1:])[1]
            print(f"{os.path.basename(SO)} rank {k} {side:5s} rows={n:7d} mode {mode} {names[mode]:11s} {t:8.3f} ms"
                  f"  {1e6 * t / max(n, 1):8.2f} ns/row", flush=True)


if __name__ == "__main__":
    main()
