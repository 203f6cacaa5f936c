"""Dev (GPU box, under rocprofv3): one top-10 and one top-100 call on a sample of
the configs[3] factors after two iterations (counter passes of the product kernel).
    python tools/ab/topk_once.py [sample_users]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    for top in (10, 100):
        E.topk_rows(Q, s, core.V, core.n_items, 128, top)
        torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
