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


def row_len_buckets(indptr, err_rows, edges=(32, 128, 512, 2048)):
    """Max per-row relative error bucketed by row length (ratings per row):
    {"<=32": e, "33-128": e, ..., ">2048": e} (">2048" = heavy rows, chunked)."""
    deg = np.diff(np.asarray(indptr))
    lo = 0
    out = {}
    for hi in list(edges) + [None]:
        sel = deg > lo if hi is None else (deg > lo) & (deg <= hi)
        name = f">{lo}" if hi is None else (f"<={hi}" if lo == 0 else f"{lo + 1}-{hi}")
        out[name] = {"rows": int(sel.sum()), "max_rel_err": float(err_rows[sel].max()) if sel.any()
                     else None}
        lo = hi if hi is not None else lo
    return out


def rel_row_errs(x, ref):
    """Per-row ||x - ref|| / ||ref|| (vector)."""
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    return np.linalg.norm(x - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-6)


def report(name, value):
    """Append a measured error to $ALS_TEST_REPORT (JSON lines) when set."""
    import json
    import os
    path = os.environ.get("ALS_TEST_REPORT")
    if path:
        with open(path, "a") as f:
            v = value if isinstance(value, (dict, list)) else float(value)
            f.write(json.dumps({"test": name, "value": v}) + "\n")


def oracle_train_c(users, items, ratings, rank, iterations, reg, U0, implicit=False, alpha=1.0):
    """ALS.train restated (oracle.als_oracle's loop) with the C half-sweeps
    (oracle/als_oracle.c, OpenMP) for the larger parity cases.
    Returns (U, V, umap, imap, uids, iids)."""
    from oracle import als_oracle as O
    from oracle import c_oracle as C
    users = np.asarray(users, np.int64)
    items = np.asarray(items, np.int64)
    ratings = np.asarray(ratings, np.float32)
    umap, uids = O.index_build(users, int(users.max()) + 1)
    imap, iids = O.index_build(items, int(items.max()) + 1)
    ip = O.csr_build(imap[items], umap[users], ratings, len(iids))
    up = O.csr_build(umap[users], imap[items], ratings, len(uids))
    U = np.asarray(U0, np.float32)
    V = np.zeros((len(iids), rank), np.float32)
    for _ in range(iterations):
        V, st = C.half_sweep(*ip, U, reg, implicit=implicit, alpha=alpha)
        assert not st.any()
        U, st = C.half_sweep(*up, V, reg, implicit=implicit, alpha=alpha)
        assert not st.any()
    return U, V, umap, imap, uids, iids
