"""CPU tests of the oracle itself (no GPU): pin it before trusting it.

* computeError against the reference's own known answers (output.txt:16-18).
* The numpy restatement against the independent C restatement of Spark's packed
  dspr + dppsv arithmetic (oracle/als_oracle.c), explicit and implicit.
* K1 / schedule / top-k oracle functions against brute force.
"""
import json
import os

import numpy as np
import pytest

from oracle import als_oracle as O
from oracle import c_oracle as C
from helpers import planted, rel_row_err

HERE = os.path.dirname(os.path.abspath(__file__))


def test_compute_error_known_answers():
    kat = json.load(open(os.path.join(HERE, "golden", "compute_error_kat.json")))
    assert len(kat["cases"]) == 3
    for case in kat["cases"]:
        got = O.compute_error(case["predicted"], case["actual"])
        # output.txt prints str(float) of Python 2: 12 significant digits
        assert float("%.12g" % got) == case["expected"], case["name"]


def test_compute_error_join_semantics():
    # duplicate keys cross-multiply like an RDD join; unmatched keys drop out
    pred = [(1, 1, 2.0), (1, 1, 4.0), (9, 9, 1.0)]
    act = [(1, 1, 3.0), (2, 2, 5.0)]
    assert O.compute_error(pred, act) == pytest.approx(1.0)


def test_get_ratings_tuple_matches_output_txt():
    # output.txt:2 shows the parsed form of ratings.dat lines
    assert O.get_ratings_tuple("1::1193::5::978300760") == (1, 1193, 5.0)
    assert O.get_ratings_tuple("1::914::3::978301968") == (1, 914, 3.0)


def test_index_and_csr_oracle_bruteforce():
    rng = np.random.default_rng(0)
    ids = rng.integers(0, 500, 3000)
    mp, uniq = O.index_build(ids, 600)
    assert np.array_equal(uniq, np.unique(ids))
    assert np.all(mp[uniq] == np.arange(len(uniq)))
    assert np.all(mp[np.setdiff1d(np.arange(600), uniq)] == -1)
    rows = mp[ids]
    cols = rng.integers(0, 50, 3000).astype(np.int32)
    vals = rng.random(3000).astype(np.float32)
    ptr, idx, val = O.csr_build(rows, cols, vals, len(uniq))
    for r in range(len(uniq)):
        sel = np.nonzero(rows == r)[0]  # input order within the row (stable)
        assert np.array_equal(idx[ptr[r]:ptr[r + 1]], cols[sel])
        assert np.array_equal(val[ptr[r]:ptr[r + 1]], vals[sel])


def test_schedule_oracle_covers_every_rating_once():
    deg = np.array([0, 5, 300, 64, 65, 1000, 1])
    ptr = np.concatenate([[0], np.cumsum(deg)])
    light, heavy, slot_begin, chunks = O.schedule_build(ptr, 64)
    assert sorted(np.concatenate([light, heavy]).tolist()) == list(range(len(deg)))
    assert list(deg[light]) == sorted(deg[light], reverse=True)  # LPT order
    covered = np.zeros(ptr[-1], int)
    for r, b, e in chunks:
        assert e - b <= 64 and ptr[r] <= b < e <= ptr[r + 1]
        covered[b:e] += 1
    for r in heavy:
        assert covered[ptr[r]:ptr[r + 1]].min() == 1
    assert slot_begin[-1] == len(chunks)


@pytest.mark.parametrize("rank", [1, 4, 10, 33, 64])
@pytest.mark.parametrize("implicit", [False, True])
def test_numpy_oracle_matches_c_restatement(rank, implicit):
    u, i, r = planted(150, 90, density=0.1, seed=rank, dup=10)
    if implicit:
        r = (r - 2.5).astype(np.float32)
    mu, _ = O.index_build(u, int(u.max()) + 1)
    mi, _ = O.index_build(i, int(i.max()) + 1)
    ptr, idx, val = O.csr_build(mi[i], mu[u], r, int(mi.max()) + 1)
    Y = O.initialize(int(mu.max()) + 1, rank, seed=rank)
    X_np = O.half_sweep(ptr, idx, val, Y, 0.1, implicit, 3.0)
    X_c, st = C.half_sweep(ptr, idx, val, Y, 0.1, implicit, 3.0, threads=2)
    assert st.max() == 0
    assert rel_row_err(X_c, X_np) < 1e-9


def test_c_oracle_reports_failed_cholesky():
    # a row whose normal equations are singular (reg = 0, one rating, rank 4)
    ptr = np.array([0, 1], np.int64)
    X, st = C.half_sweep(ptr, np.array([0], np.int32), np.array([3.0], np.float32),
                         np.array([[1, 0, 0, 0]], np.float32), 0.0)
    assert st[0] == 2  # dpptrf info: column 2 is not positive


def test_yty_oracle_matches_c():
    Y = np.random.default_rng(1).standard_normal((1000, 12)).astype(np.float32)
    up = C.yty_packed_upper(Y)
    full = np.zeros((12, 12))
    for j in range(12):
        for ii in range(j + 1):
            full[ii, j] = full[j, ii] = up[j * (j + 1) // 2 + ii]
    assert np.allclose(full, O.yty(Y), rtol=1e-12, atol=1e-9)


def test_topk_oracle_bruteforce_and_ties():
    rng = np.random.default_rng(3)
    Q = rng.standard_normal((20, 5)).astype(np.float32)
    V = rng.standard_normal((50, 5)).astype(np.float32)
    V[7] = V[3]
    idx, sc = O.topk(Q, V, 8)
    S = Q.astype(np.float64) @ V.astype(np.float64).T
    for q in range(20):
        order = sorted(range(50), key=lambda j: (-S[q, j], j))[:8]
        assert list(idx[q]) == order
    idx2, _ = O.topk(Q, V[:5], 8)
    assert np.all(idx2[:, 5:] == -1)


def test_train_oracle_converges_on_planted_data():
    u, i, r = planted(300, 200, density=0.1, seed=4)
    U, V, umap, imap, _, _ = O.train(u, i, r, rank=8, iterations=8, reg=0.1, seed=5)
    sse, n = O.rmse(U, V, umap, imap, u, i, r)
    assert n == len(u)
    assert np.sqrt(sse / n) < 0.85  # planted noise sd is 0.8 (+ rounding)
