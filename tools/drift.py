"""Dev tool (CPU only): is the configs[0] fit-level drift ALS's own sensitivity?

The GPU fit at configs[0] (ml-latest-small shape, rank 10, lambda 0.1) drifts from the
fp64 oracle from ~1e-6 per row after one iteration to ~3.5e-5 after 10 and ~4.2e-5 after
20 (tests/test_gpu_configs.py::test_configs0_full_fit_per_iteration, profiles/r05/
errors_final.jsonl), while one half-sweep from identical inputs is ~1e-6.  This runs the
C restatement of Spark's per-row arithmetic (oracle/als_oracle.c: fp64 dspr + dppsv, fp32
factors in and out, as Spark's Float factor arrays) three ways from the same start:

  ref      the oracle;
  init     the oracle from U0 perturbed once by `eps` relative per row (a random direction);
  noise    the oracle with every half-sweep's output perturbed by `eps` relative per row
           (a fresh random direction each time): an unbiased solver whose per-half-sweep
           error is `eps` — the GPU's measured per-half-sweep error is ~1e-6;
  fp32     (--fp32) a textbook fp32 solver: numpy fp32 Gram accumulated rating by
           rating, fp32 Cholesky (LAPACK spotrf) — what any fp32 ALS would do;

and prints, per iteration, the max over rows of ||x - x_ref|| / ||x_ref|| of each.  If
`noise` tracks the GPU curve, the drift is the ALS map's own amplification of
per-step rounding, not a bias in the kernels.

    python tools/drift.py [iters] [eps] [seed] [--fp32]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _pkgload  # noqa: E402

_pkgload.load()
import torch  # noqa: E402

import als_mi355x.datasets as D  # noqa: E402
from oracle import als_oracle as O  # noqa: E402
from oracle import c_oracle as C  # noqa: E402


def rel(x, ref):
    x, ref = np.asarray(x, np.float64), np.asarray(ref, np.float64)
    return float((np.linalg.norm(x - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-6)).max())


def perturb(x, eps, rng):
    d = rng.standard_normal(x.shape)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return (x + eps * np.linalg.norm(x, axis=1, keepdims=True) * d).astype(np.float32)


def half_sweep_fp32(indptr, indices, vals, Y, reg):
    """Spark's normal equations and Cholesky, every operation in fp32."""
    n, k = len(indptr) - 1, Y.shape[1]
    X = np.zeros((n, k), np.float32)
    for row in range(n):
        a, b = indptr[row], indptr[row + 1]
        Ys = Y[indices[a:b]].astype(np.float32)
        A = np.zeros((k, k), np.float32)
        rhs = np.zeros(k, np.float32)
        for j in range(b - a):
            A += np.outer(Ys[j], Ys[j]).astype(np.float32)
            rhs += (vals[a + j] * Ys[j]).astype(np.float32)
        A[np.diag_indices(k)] += np.float32(reg * (b - a))
        L = np.linalg.cholesky(A)
        X[row] = np.linalg.solve(L.T, np.linalg.solve(L, rhs)).astype(np.float32)
    return X


def main():
    fp32 = "--fp32" in sys.argv
    sys.argv = [a for a in sys.argv if a != "--fp32"]
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    eps = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-6
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    u, i, r = (t.numpy() for t in D.synthetic_config("ml_latest_small", device="cpu"))
    rank, reg = 10, 0.1
    umap, uids = O.index_build(u, int(u.max()) + 1)
    imap, iids = O.index_build(i, int(i.max()) + 1)
    ip = O.csr_build(imap[i], umap[u], r, len(iids))
    up = O.csr_build(umap[u], imap[i], r, len(uids))
    g = torch.Generator().manual_seed(5)
    U0 = torch.randn((len(uids), rank), generator=g)
    U0 = (U0 / U0.norm(dim=1, keepdim=True)).numpy().astype(np.float32)
    rng = np.random.default_rng(seed)
    U = {"ref": U0, "init": perturb(U0, eps, rng), "noise": U0}
    if fp32:
        U["fp32"] = U0
    out = []
    for it in range(iters):
        V = {}
        for key in U:
            if key == "fp32":
                V[key] = half_sweep_fp32(*ip, U[key], reg)
                U[key] = half_sweep_fp32(*up, V[key], reg)
                continue
            V[key], st = C.half_sweep(*ip, U[key], reg)
            assert not st.any()
            if key == "noise":
                V[key] = perturb(V[key], eps, rng)
            U[key], st = C.half_sweep(*up, V[key], reg)
            assert not st.any()
            if key == "noise":
                U[key] = perturb(U[key], eps, rng)
        row = {"iteration": it + 1}
        for key in [k_ for k_ in U if k_ != "ref"]:
            row[key] = [rel(V[key], V["ref"]), rel(U[key], U["ref"])]
        out.append(row)
        print(json.dumps(row))
    return out


if __name__ == "__main__":
    main()
