"""Dev (GPU box): top-k time per (query, item) pair against the V size, on the
configs[3] factors after two iterations: does the sweep slow down once the split
V table outgrows the Infinity Cache?
    python tools/topk_vsize.py [sample_users]"""
import os
import sys

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
    for top in (10, 100):
        for n_v in (1000000, 500000, 250000, 125000):
            V = core.V[:n_v].contiguous()
            E.topk_rows(Q, s, V, n_v, 128, top)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            E.topk_rows(Q, s, V, n_v, 128, top)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            print(f"top{top} n_v {n_v}: {ms:.1f} ms  {1e6 * ms / (s * n_v):.3f} ps/pair "
                  f"(hi plane {n_v * 256 / 2**20:.0f} MiB)", flush=True)


if __name__ == "__main__":
    main()
