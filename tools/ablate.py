"""Dev tool: time the phases of the light-row half-sweep kernel on the ML-25M-shaped
synthetic data (see tools/dev_ablate.hip).  Run on the GPU box:
    python tools/ablate.py
Prints ms per launch for each mode on the item side and the user side."""
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

SO = os.environ.get("ALS_DEV_SO", os.path.join(ROOT, "tools", "libals_dev.so"))


def build():
    src = os.path.join(ROOT, "tools", "dev_ablate.hip")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-shared", "--offload-arch=gfx950",
                           "-std=c++17", src, "-o", SO])


def split_table(Y, k):
    """The explicit path's split table (as split_table_kernel): hi | lo << 16 of 2^ey * Y."""
    ey = 14 - math.floor(math.log2(float(Y[:, :k].abs().max())))
    t = Y[:, :k].float() * (2.0 ** ey)
    hi = t.half()
    lo = (t - hi.float()).half()
    w = (hi.view(torch.int16).to(torch.int32) & 0xFFFF) | (lo.view(torch.int16).to(torch.int32) << 16)
    z = torch.zeros((1, k), dtype=torch.int32, device=Y.device)
    return torch.cat([w, z]).contiguous(), ey


def main():
    if "--build" in sys.argv:
        build()
        return
    L = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    F = ctypes.c_float
    L.dev_ablate.argtypes = [ctypes.c_int, P, P, P, P, ctypes.c_int, P, ctypes.c_int, F, F, F, P,
                             ctypes.c_int, F, P, P]
    L.dev_ablate_wg.argtypes = L.dev_ablate.argtypes
    L.dev_ablate_w1.argtypes = L.dev_ablate.argtypes
    wg = "--wg" in sys.argv
    w1 = "--w1" in sys.argv
    k = 128 if (wg or w1) else 64
    fn = L.dev_ablate_w1 if w1 else (L.dev_ablate_wg if wg else L.dev_ablate)
    modes = (0, 1, 2) if (wg or w1) else (0, 1, 2, 5)
    dev = torch.device("cuda", 0)
    u, i, r = D.synthetic_config("ml25m", device=dev)
    core = E.ALSCore(u, i, r, device=dev)
    core.init_factors(k, seed=5)
    core.iterate(0.1)
    torch.cuda.synchronize()
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    names = {0: "full (tile LDL)", 1: "gram only", 2: "solve only (tile LDL)",
             5: "half gram / half solve"}
    for side, blk, Y, X in (("item", core.item_block, core.U, core.V),
                            ("user", core.user_block, core.V, core.U)):
        X2 = torch.empty_like(X)
        Ysp, ey = split_table(Y, k)
        er = 14 - math.floor(math.log2(float(blk.val.abs().max())))
        sc = (Y.shape[0], 2.0 ** er, 2.0 ** (-2 * ey), 2.0 ** (-ey - er))
        col = blk.col
        if "--local-cols" in sys.argv:
            # every gather hits the first 64 rows of Y (L2-resident): isolates gather latency
            col = (blk.col & 63).contiguous()
        for mode in modes:
            times = []
            for rep in range(4):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = fn(mode, blk.row_ptr.data_ptr(), col.data_ptr(),
                                  blk.val.data_ptr(), blk.light_rows.data_ptr(), blk.n_light,
                                  Ysp.data_ptr(), *sc, X2.data_ptr(), k, 0.1, st.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0
                times.append(e0.elapsed_time(e1))
            t = sorted(times[1:])[1]
            print(f"{side:5s} rows={blk.n_light:7d} mode {mode} {names[mode]:24s} {t:8.3f} ms"
                  f"  {1e6 * t / blk.n_light:8.2f} ns/row", flush=True)


if __name__ == "__main__":
    main()
