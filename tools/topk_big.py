"""Dev: configs[4] top-10 / top-100 timing on configs[3]-shaped factors (2 ALS
iterations from the seed), for the library ALS_HIP_LIB points at (with ALS_HIP_DEV=1).
    python tools/topk_big.py [sample]
TOPK_SAVE=f.pt: save the results; TOPK_CMP=f.pt: print the agreement with saved ones."""
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
    ml = len(sys.argv) > 1 and sys.argv[1] == "ml25m"  # configs[1] shape, rank 64, all users
    s = 0 if ml else (int(sys.argv[1]) if len(sys.argv) > 1 else 262144)
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
    from als_mi355x import _lib as _L
    lib = _L.LIB_PATH  # the library actually loaded (ALS_HIP_LIB counts only with ALS_HIP_DEV=1)
    res = {}
    for top in (10, 100):
        res[top] = E.topk_rows(Q, s, core.V, core.n_items, k, top)
        torch.cuda.synchronize()
        L = E._lib.lib()
        cnt = hasattr(L, "als_dev_tk_counters")
        if cnt:
            import ctypes
            buf = (ctypes.c_ulonglong * 8)()
            L.als_dev_tk_counters(buf, 1)
        ts = []
        for _ in range(2):
            t0 = time.perf_counter()
            E.topk_rows(Q, s, core.V, core.n_items, k, top)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"{lib} top{top}: {1e3 * min(ts):.1f} ms  {s / min(ts) / 1e6:.3f} M recs/s", flush=True)
        if cnt:
            L.als_dev_tk_counters(buf, 1)
            print(f"  counters per call: {[v // 2 for v in buf[:5]]}", flush=True)
    keep = 1 << 20  # rows saved / compared (all rows would be 8.8 GB at 10M users)
    if os.environ.get("TOPK_SAVE"):
        torch.save({t: tuple(x[:keep].cpu() for x in r) for t, r in res.items()},
                   os.environ["TOPK_SAVE"])
    if os.environ.get("TOPK_CMP"):
        ref = torch.load(os.environ["TOPK_CMP"], weights_only=True)
        for t, r in res.items():
            i0, s0 = ref[t]
            i1, s1 = (x[:keep].cpu() for x in r)
            print(f"{lib} top{t}: index agreement {float((i0 == i1).float().mean()):.7f} "
                  f"max|dscore| {float((s0 - s1).abs().max()):.3e}", flush=True)


if __name__ == "__main__":
    main()
