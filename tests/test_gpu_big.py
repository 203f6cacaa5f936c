"""GPU parity at BASELINE.json configs[3] and configs[4] — the 1e9-rating workload.

configs[3]: the 1e9-rating power-law synthetic (10M users x 1M items, rank 128,
explicit, regParam 0.1) that bench.py times, built by the same device generator
(datasets.big_config) into the single-GPU engine with the production chunk.  One
item half-sweep from the seeded U, then one user half-sweep from the GPU's V,
each compared on a row sample with the C restatement of Spark's dspr + dppsv
(oracle/als_oracle.c) from identical source factors:
  * items: the 50 heaviest (1M-5M ratings each: ~500-2,500 fp32 chunk partials
    summed in fp64 per row) and 5,000 uniformly drawn items;
  * users: the 50 heaviest (the chunked heavy user rows) and 20,000 drawn users.
Bar: 1e-4 relative per row (north_star), errors reported by row length.

configs[4]: recommendForAllUsers top-10 and top-100 over ALL 10M users x 1M items
on the configs[3] factors after two iterations.  Full size: size-independent
properties on every row (scores descending, indices valid and distinct per
row, scores = fp64 dot products within 1e-5 on a sample of entries); a
1,000-user sample against the fp64 oracle over all 1M items: item indices
identical except where scores tie within 1e-5.

Reference call sites: RecommenderSystem.py:148-150 (ALS.train / predictAll),
:229-247 (predict over unrated movies + takeOrdered(20)).
"""
import numpy as np
import pytest
import torch

import als_mi355x.datasets as D
import als_mi355x.engine as E
from helpers import rel_row_errs, report, row_len_buckets
from oracle import als_oracle as O
from oracle import c_oracle as C

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-4
RANK = 128
REG = 0.1
EDGES = (32, 128, 512, 2048, 100_000, 1_000_000)


@pytest.fixture(scope="module")
def big():
    u, i, r = D.big_config("big1b", device=DEV)
    core = E.ALSCore(u, i, r, device=DEV)
    del u, i, r
    torch.cuda.empty_cache()
    assert core.nnz == 1_000_000_000
    core.init_factors(RANK, seed=5)
    return core


def _sub_csr(block, rows: np.ndarray):
    """Host CSR (indptr, col, val) of the given dense rows of a device CSR side."""
    r = torch.as_tensor(rows, device=DEV, dtype=torch.int64)
    beg, end = block.row_ptr[r], block.row_ptr[r + 1]
    deg = end - beg
    ptr = torch.zeros(len(rows) + 1, dtype=torch.int64, device=DEV)
    ptr[1:] = torch.cumsum(deg, 0)
    rid = torch.repeat_interleave(torch.arange(len(rows), device=DEV), deg)
    pos = beg[rid] + (torch.arange(int(ptr[-1]), device=DEV) - ptr[:-1][rid])
    out = ptr.cpu().numpy(), block.col[pos].cpu().numpy(), block.val[pos].cpu().numpy()
    del rid, pos
    return out


def _sample(block, n_heavy, n_rand, seed):
    deg = block.row_ptr[1:] - block.row_ptr[:-1]
    heavy = torch.topk(deg, n_heavy).indices.cpu().numpy()
    rnd = np.random.default_rng(seed).choice(block.n_rows, n_rand, replace=False)
    return np.unique(np.concatenate([heavy, rnd])), heavy, deg


def _check_half(core, block, rows, Y_host, X_dev, tag):
    ptr, col, val = _sub_csr(block, rows)
    X_ref, st = C.half_sweep(ptr, col, val, Y_host, REG)
    assert not st.any()
    X = X_dev[torch.as_tensor(rows, device=DEV)].cpu().numpy()
    assert np.all(X[:, RANK:] == 0.0)
    err = rel_row_errs(X[:, :RANK], X_ref)
    buckets = row_len_buckets(ptr, err, EDGES)
    report(tag, buckets)
    assert err.max() <= TOL, buckets
    return ptr


def test_configs3_item_half_sweep(big):
    core = big
    U0 = core.U[:, :RANK].cpu().numpy()
    core.status.zero_()
    core.half_sweep_items(REG)
    torch.cuda.synchronize()
    core.check_status()
    rows, heavy, deg = _sample(core.item_block, 50, 5000, 11)
    # the heavy head really is the many-hundred-chunk regime
    hdeg = deg[torch.as_tensor(heavy, device=DEV)]
    ch = core.item_block.chunk
    assert int(hdeg.max()) > 150 * ch and int(hdeg.min()) > 25 * ch
    report("configs3_item_chunks", {"n_chunks": core.item_block.n_chunks,
                                    "heaviest_50_ratings": [int(hdeg.min()), int(hdeg.max())]})
    _check_half(core, core.item_block, rows, U0, core.V, "configs3_item_half_sweep_by_row_length")


def test_configs3_user_half_sweep(big):
    core = big
    V0 = core.V[:, :RANK].cpu().numpy()  # the GPU's item factors: identical source factors
    core.status.zero_()
    core.half_sweep_users(REG)
    torch.cuda.synchronize()
    core.check_status()
    rows, heavy, deg = _sample(core.user_block, 50, 20000, 12)
    # chunked heavy user rows, where the data has rows past the production chunk, are in
    # the sample (_sample takes the longest rows)
    assert core.user_block.n_heavy > 0 or int(deg.max()) <= core.user_block.chunk
    _check_half(core, core.user_block, rows, V0, core.U, "configs3_user_half_sweep_by_row_length")


@pytest.mark.parametrize("top", [10, 100])
def test_configs4_topk_all_users(big, top):
    core = big
    if top == 10:
        core.iterate(REG)  # the factors of two full iterations (the user half above + this)
        torch.cuda.synchronize()
        core.check_status()
    n_u, n_i = core.n_users, core.n_items
    idx, sc = E.topk_rows(core.U, n_u, core.V, n_i, RANK, top)
    torch.cuda.synchronize()
    # full-size properties on every row
    assert bool((idx >= 0).all()) and bool((idx < n_i).all())
    assert bool((sc[:, :-1] >= sc[:, 1:]).all())
    srt = torch.sort(idx, dim=1).values
    assert bool((srt[:, 1:] != srt[:, :-1]).all())
    del srt
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    rr = torch.randint(0, n_u, (200_000,), device=DEV, generator=g)
    pp = torch.randint(0, top, (200_000,), device=DEV, generator=g)
    ii = idx[rr, pp].long()
    dot = (core.U[rr, :RANK].double() * core.V[ii, :RANK].double()).sum(1)
    s = sc[rr, pp].double()
    assert bool(((s - dot).abs() <= 1e-5 * dot.abs().clamp(min=1.0)).all())
    # sample vs the fp64 oracle over all 1M items
    rows = np.sort(np.random.default_rng(13).choice(n_u, 1000, replace=False))
    U = core.U[torch.as_tensor(rows, device=DEV), :RANK].cpu().numpy()
    V = core.V[:, :RANK].cpu().numpy()
    ref_i, ref_s = O.topk(U, V, top)
    got_i = idx[torch.as_tensor(rows, device=DEV)].cpu().numpy()
    got_s = sc[torch.as_tensor(rows, device=DEV)].cpu().numpy()
    del idx, sc
    Vd = V.astype(np.float64)
    swaps = 0
    for t in range(len(rows)):
        bad = np.nonzero(got_i[t] != ref_i[t])[0]
        if len(bad):
            S = Vd[got_i[t, bad]] @ U[t].astype(np.float64)
            for p, s_got in zip(bad, S):
                swaps += 1
                assert abs(s_got - ref_s[t, p]) <= 1e-5 * max(1.0, abs(ref_s[t, p])), (t, p)
    np.testing.assert_allclose(got_s, ref_s, rtol=1e-5, atol=1e-5)
    report(f"configs4_top{top}_sample_tie_swaps", {"rows": len(rows), "swaps": swaps})
