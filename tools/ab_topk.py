"""Dev A/B timing of recommendForAll variants (NOT the bench): the configs[3] factors
after two ALS iterations (10M users x 1M items, rank 128), top-10 and top-100 for a
262,144-user prefix (or all users with --all), with the library named by ALS_HIP_LIB (+ ALS_HIP_DEV=1; a
tools/ab/variant.py build) or the product one; a 64-user sample is checked against
the fp64 oracle (identical except fp64 ties within 1e-5).
    ALS_HIP_LIB=tools/ab/libals_x.so python tools/ab_topk.py [--all]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import _pkgload  # noqa: E402

_pkgload.load()
from als_mi355x import datasets as D, engine as E  # noqa: E402
from als_mi355x import _lib as _L  # noqa: E402


def _lib_loaded():
    """The library actually loaded (ALS_HIP_LIB counts only with ALS_HIP_DEV=1)."""
    return _L.LIB_PATH
from oracle import als_oracle as O  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    u, i, r = D.big_config("big1b", device=dev)
    core = E.ALSCore(u, i, r, device=dev)
    del u, i, r
    torch.cuda.empty_cache()
    k = 128
    core.init_factors(k, seed=5)
    for _ in range(2):
        core.iterate(0.1)
    torch.cuda.synchronize()
    n_q = core.n_users if "--all" in sys.argv else 262_144
    out = {"lib": _lib_loaded(), "n_q": n_q}
    V = core.V[:, :k].cpu().numpy()
    rows = np.arange(0, n_q, n_q // 64)[:64]
    for top in (10, 100):
        E.topk_rows(core.U, 65536, core.V, core.n_items, k, top)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        idx, sc = E.topk_rows(core.U, n_q, core.V, core.n_items, k, top)
        b.record()
        torch.cuda.synchronize()
        out[f"top{top}_ms"] = round(a.elapsed_time(b), 3)
        Uq = core.U[torch.as_tensor(rows, device=dev), :k].cpu().numpy()
        ref_i, ref_s = O.topk(Uq, V, top)
        gi = idx[torch.as_tensor(rows, device=dev)].cpu().numpy()
        gs = sc[torch.as_tensor(rows, device=dev)].cpu().numpy()
        bad = 0
        for t in range(len(rows)):
            for p in np.nonzero(gi[t] != ref_i[t])[0]:
                s_got = float(V[gi[t, p]].astype(np.float64) @ Uq[t].astype(np.float64))
                if abs(s_got - ref_s[t, p]) > 1e-5 * max(1.0, abs(ref_s[t, p])):
                    bad += 1
        out[f"top{top}_bad"] = bad
        out[f"top{top}_score_err"] = float(np.abs(gs - ref_s).max())
        del idx, sc
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
