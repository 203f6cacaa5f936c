"""Dev ablation (GPU box) of topk_split_kernel on the configs[3] factors after two
iterations: mode 0 = product, 1 = scores only, 2 = filter against an unbeatable
threshold (no list work), 3 = product filter counting offers.  Uses
tools/libals_topk_dev.so (tools/dev_topk.hip, the product topk.hip + dev modes).
    python tools/ab/topk_modes.py [sample_users]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import _pkgload  # noqa: E402

_pkgload.load()
from als_mi355x import _lib, datasets as D, engine as E  # noqa: E402


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
    n_v = core.n_items
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libals_topk_dev.so"))
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    L.dev_topk.argtypes = [ctypes.c_int, P, I64, P, I64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           P, P, P, ctypes.c_size_t, P, P]
    for top in (10, 100):
        ws = torch.empty(int(_lib.lib().als_topk_workspace_bytes(s, n_v, 128, top)),
                         dtype=torch.uint8, device=dev)
        idx = torch.empty((s, top), dtype=torch.int32, device=dev)
        sc = torch.empty((s, top), dtype=torch.float32, device=dev)
        dbg = torch.zeros(s * 8 + 64, dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        for mode in (0, 1, 2, 4, 5, 3, 0):
            args = (mode, Q.data_ptr(), s, core.V.data_ptr(), n_v, Q.shape[1], 128, top,
                    idx.data_ptr(), sc.data_ptr(), ws.data_ptr(), ws.numel(), dbg.data_ptr(), st)
            assert L.dev_topk(*args) == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert L.dev_topk(*args) == 0
            e1.record()
            torch.cuda.synchronize()
            extra = ""
            if mode == 3:
                rg = 2 if top <= 16 else 1
                waves = (s + 128 * rg - 1) // (128 * rg) * 8
                cnt = dbg[:waves].double()
                til = dbg[waves:2 * waves].double()
                vt = 128
                extra = (f" refined blocks/wave mean {float(cnt.mean()):.0f} of "
                         f"{(n_v + 15) // 16} blocks; tiles/wave mean {float(til.mean()):.0f} "
                         f"min {float(til.min()):.0f} max {float(til.max()):.0f} of "
                         f"{(n_v + vt - 1) // vt}")
            print(f"top{top} mode {mode}: {e0.elapsed_time(e1):.1f} ms{extra}", flush=True)


if __name__ == "__main__":
    main()
