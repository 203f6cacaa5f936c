"""Seeded synthetic rating sets for tests (planted low-rank model, SURVEY §8d shape rules)."""
import numpy as np


def planted(n_users, n_items, density=0.05, k_true=8, seed=0, heavy_items=(), heavy_users=(),
            half_stars=True, dup=0, id_gap=1):
    """Return (users, items, ratings) int32/int32/float32 with optional heavy rows,
    duplicate (u,i) pairs (`dup` extra copies) and sparse ids (ids multiplied by id_gap)."""
    rng = np.random.default_rng(seed)
    mask = rng.random((n_users, n_items)) < density
    for i in heavy_items:
        mask[:, i] = True
    for u in heavy_users:
        mask[u, :] = True
    mask[np.arange(n_users), rng.integers(0, n_items, n_users)] = True  # every user rates
    mask[rng.integers(0, n_users, n_items), np.arange(n_items)] = True  # every item rated
    u, i = np.nonzero(mask)
    perm = rng.permutation(len(u))
    u, i = u[perm], i[perm]
    us = rng.normal(0, 0.35, (n_users, k_true))
    vs = rng.normal(0, 0.35, (n_items, k_true))
    r = 3.6 + (us[u] * vs[i]).sum(1) + rng.normal(0, 0.8, len(u))
    r = np.round(r * 2) / 2 if half_stars else np.round(r)
    r = np.clip(r, 0.5 if half_stars else 1, 5)
    if dup:
        sel = rng.integers(0, len(u), dup)
        u = np.concatenate([u, u[sel]])
        i = np.concatenate([i, i[sel]])
        r = np.concatenate([r, np.clip(r[sel] - 1, 0.5, 5)])
    return (u * id_gap).astype(np.int32), (i * id_gap).astype(np.int32), r.astype(np.float32)


def rel_row_err(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    num = np.linalg.norm(x - ref, axis=1)
    den = np.maximum(np.linalg.norm(ref, axis=1), 1e-6)
    return float((num / den).max())


def report(name, value):
    """Append a measured error to $ALS_TEST_REPORT (JSON lines) when set."""
    import json
    import os
    path = os.environ.get("ALS_TEST_REPORT")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"test": name, "value": float(value)}) + "\n")
