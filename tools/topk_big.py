"""Dev: configs[4] top-10 / top-100 timing on configs[3]-shaped factors (2 ALS
iterations from the seed), for the library ALS_HIP_LIB points at (with ALS_HIP_DEV=1).
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
