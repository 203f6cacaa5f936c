"""GPU parity tests: each HIP kernel through the C ABI vs the CPU oracle.

Bars (DESIGN.md "Parity"):
  * K1 (id maps, CSR, schedule): bit-exact.
  * K2/K3 (half-sweep factors): max over rows of ||x - x_ref|| / ||x_ref|| <= 1e-4
    against the fp64 oracle from identical source factors (north_star: 1e-4 relative).
  * K2b (YtY): relative Frobenius error <= 1e-6.
  * K4 (predict / RMSE): predictions within 1e-9 relative (fp64 dot of fp32 factors),
    RMSE within 1e-9; computeError KAT (output.txt:16-18) exact to 11 digits.
  * K5 (top-k): identical indices except where the oracle's fp64 scores tie within 1e-5.
"""
import dataclasses
import json
import math
import os

import numpy as np
import pytest
import torch

import als_mi355x.engine as E
from oracle import als_oracle as O
from helpers import planted, rel_row_err, rel_row_errs, report

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
DEV = "cuda:0"


def _t(x, dtype):
    return torch.as_tensor(np.ascontiguousarray(x)).to(DEV, dtype)


def _core(u, i, r, chunk=E.DEFAULT_CHUNK):
    return E.ALSCore(u, i, r, device=DEV, chunk=chunk)


# ---------------------------------------------------------------- K1
@pytest.mark.parametrize("n,space,seed", [(1, 1, 0), (1000, 50, 1), (50000, 7000, 2),
                                          (300000, 1 << 20, 3)])
def test_index_build_bitexact(n, space, seed):
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, space, n).astype(np.int32)
    ws = E.Workspace(DEV)
    idx = E.build_index(_t(ids, torch.int32), space, ws)
    mp, uniq = O.index_build(ids, space)
    assert idx.n == len(uniq)
    np.testing.assert_array_equal(idx.map.cpu().numpy(), mp)
    np.testing.assert_array_equal(idx.uniq.cpu().numpy(), uniq)


@pytest.mark.parametrize("kw", [dict(n_users=50, n_items=40, density=0.3),
                                dict(n_users=700, n_items=300, density=0.05, heavy_items=(3,),
                                     dup=40, id_gap=3),
                                dict(n_users=3000, n_items=2000, density=0.02, seed=5)])
def test_csr_build_bitexact(kw):
    u, i, r = planted(**kw)
    core = _core(u, i, r, chunk=64)
    umap, uids = O.index_build(u, int(u.max()) + 1)
    imap, iids = O.index_build(i, int(i.max()) + 1)
    for block, rows, cols, n in ((core.user_block, umap[u], imap[i], len(uids)),
                                 (core.item_block, imap[i], umap[u], len(iids))):
        ptr_, idx_, val_ = O.csr_build(rows, cols, r, n)
        np.testing.assert_array_equal(block.row_ptr.cpu().numpy(), ptr_)
        np.testing.assert_array_equal(block.col.cpu().numpy(), idx_)
        np.testing.assert_array_equal(block.val.cpu().numpy(), val_)
        light, heavy, slot_begin, chunks = O.schedule_build(ptr_, 64)
        assert block.n_light == len(light) and block.n_heavy == len(heavy)
        assert block.n_chunks == len(chunks)
        np.testing.assert_array_equal(block.light_rows[:len(light)].cpu().numpy(), light)
        if len(heavy):
            np.testing.assert_array_equal(block.heavy_rows[:len(heavy)].cpu().numpy(), heavy)
            np.testing.assert_array_equal(block.heavy_slot_begin.cpu().numpy(), slot_begin)
            ch = np.array(chunks)
            np.testing.assert_array_equal(block.chunk_row[:len(ch)].cpu().numpy(), ch[:, 0])
            np.testing.assert_array_equal(block.chunk_begin[:len(ch)].cpu().numpy(), ch[:, 1])
            np.testing.assert_array_equal(block.chunk_end[:len(ch)].cpu().numpy(), ch[:, 2])


# ---------------------------------------------------------------- K2/K3
@pytest.mark.parametrize("rank", [1, 4, 8, 10, 12, 16, 20, 32, 48, 64, 65, 100, 128])
@pytest.mark.parametrize("implicit", [False, True])
def test_half_sweep_parity(rank, implicit):
    u, i, r = planted(600, 400, density=0.04, heavy_items=(7, 11), heavy_users=(5,), seed=rank,
                      dup=25)
    if implicit:  # implicit data: include non-positive preferences (Spark: |r| confidence)
        r = (r - 2.5).astype(np.float32)
    core = _core(u, i, r, chunk=128)  # forces heavy-row chunking on the heavy rows
    alpha, reg = 4.0, 0.1
    core.init_factors(rank, seed=3)
    U0 = core.U[:, :rank].cpu().numpy()
    core.half_sweep_items(reg, implicit, alpha)
    torch.cuda.synchronize()
    assert int(core.status.item()) == 0
    ib = core.item_block
    V_ref = O.half_sweep(ib.row_ptr.cpu().numpy(), ib.col.cpu().numpy(), ib.val.cpu().numpy(),
                         U0, reg, implicit, alpha)
    V = core.V.cpu().numpy()
    assert np.all(V[:, rank:] == 0.0)
    ev = rel_row_err(V[:, :rank], V_ref)
    report(f"half_sweep_items[rank={rank},implicit={implicit}]", ev)
    assert ev <= 1e-4
    # and the user side from the oracle's V (identical source factors)
    core.V[:, :rank] = torch.as_tensor(V_ref).to(DEV)
    core.half_sweep_users(reg, implicit, alpha)
    ub = core.user_block
    U_ref = O.half_sweep(ub.row_ptr.cpu().numpy(), ub.col.cpu().numpy(), ub.val.cpu().numpy(),
                         V_ref, reg, implicit, alpha)
    eu = rel_row_err(core.U[:, :rank].cpu().numpy(), U_ref)
    report(f"half_sweep_users[rank={rank},implicit={implicit}]", eu)
    assert eu <= 1e-4


@pytest.mark.parametrize("rscale,yscale,rank", [(1e3, 1.0, 16), (1e-3, 1.0, 16), (1.0, 1e4, 16),
                                                (1.0, 1e-4, 64), (0.0, 1.0, 16), (-1.0, 1.0, 100)])
def test_half_sweep_scale_extremes(rscale, yscale, rank):
    """The split-f16 Gram scales its operands by powers of two from max|Y| and max|r|
    (computed on the device per call): parity must hold far from unit magnitudes, for
    negative ratings and for all-zero ratings (x = 0)."""
    u, i, r = planted(400, 300, density=0.05, heavy_items=(3,), seed=17)
    r = (r * rscale).astype(np.float32)
    core = _core(u, i, r, chunk=128)
    core.init_factors(rank, seed=3)
    core.U.mul_(yscale)
    U0 = core.U[:, :rank].cpu().numpy()
    reg = 0.1 * yscale * yscale  # same conditioning as at unit scale
    core.half_sweep_items(reg, False, 1.0)
    torch.cuda.synchronize()
    assert int(core.status.item()) == 0
    ib = core.item_block
    V = core.V[:, :rank].cpu().numpy()
    V_ref = O.half_sweep(ib.row_ptr.cpu().numpy(), ib.col.cpu().numpy(), ib.val.cpu().numpy(),
                         U0, reg, False, 1.0)
    if rscale == 0.0:
        assert np.all(V == 0.0) and np.all(V_ref == 0.0)
        return
    ev = rel_row_err(V, V_ref)
    report(f"half_sweep_scale[r*{rscale},y*{yscale},rank={rank}]", ev)
    assert ev <= 1e-4


@pytest.mark.parametrize("rank", [3, 16, 40, 64, 100, 128])
def test_yty_parity(rank):
    rng = np.random.default_rng(rank)
    n = 20000
    Y = rng.standard_normal((n, rank)).astype(np.float32)
    ld = E.ld_for(rank)
    Yd = torch.zeros((n, ld), dtype=torch.float32, device=DEV)
    Yd[:, :rank] = torch.as_tensor(Y).to(DEV)
    G = E.compute_yty(Yd, n, rank, E.Workspace(DEV)).cpu().numpy()
    kp = E.k_pad(rank)
    full = np.zeros((kp, kp))
    ii, jj = np.tril_indices(kp)
    full[ii, jj] = G
    full = full + np.tril(full, -1).T
    ref = O.yty(Y)
    assert np.linalg.norm(full[:rank, :rank] - ref) / np.linalg.norm(ref) <= 1e-6
    assert np.all(full[rank:, :] == 0)


def _fit_per_iteration(core, u, i, r, rank, iters, reg, implicit=False, alpha=1.0):
    """Run `iters` ALS iterations on the GPU and on the oracle from the same U0,
    comparing both factor matrices after EVERY iteration (north_star: 1e-4
    relative per iteration).  Returns (worst error, U_ref, V_ref, umap, imap)."""
    core.init_factors(rank, seed=5)
    U_ref = core.U[:, :rank].cpu().numpy().copy()
    umap, uids = O.index_build(u, int(u.max()) + 1)
    imap, iids = O.index_build(i, int(i.max()) + 1)
    ip = O.csr_build(imap[i], umap[u], r, len(iids))
    up = O.csr_build(umap[u], imap[i], r, len(uids))
    core.status.zero_()
    worst = 0.0
    for it in range(iters):
        core.iterate(reg, implicit, alpha)
        V_ref = O.half_sweep(*ip, U_ref, reg, implicit, alpha)
        U_ref = O.half_sweep(*up, V_ref, reg, implicit, alpha)
        ev = rel_row_err(core.V[:, :rank].cpu().numpy(), V_ref)
        eu = rel_row_err(core.U[:, :rank].cpu().numpy(), U_ref)
        worst = max(worst, ev, eu)
        assert max(ev, eu) <= 1e-4, f"iteration {it + 1}: item {ev:.2e}, user {eu:.2e}"
    core.check_status()
    return worst, U_ref, V_ref, umap, imap


def test_full_fit_parity_and_rmse():
    u, i, r = planted(500, 300, density=0.06, seed=11)
    rank, it, reg = 8, 5, 0.1
    core = _core(u, i, r)
    worst, U, V, umap, imap = _fit_per_iteration(core, u, i, r, rank, it, reg)
    report("full_fit_per_iteration[rank=8]", worst)
    rm, n = core.rmse(u, i, r)
    sse, n_ref = O.rmse(U, V, umap, imap, u, i, r)
    assert n == n_ref
    assert abs(rm - math.sqrt(sse / n_ref)) <= 1e-4


@pytest.mark.parametrize("rank,implicit,alpha", [(128, True, 40.0), (128, False, 1.0),
                                                (72, True, 40.0)])
def test_full_fit_parity_k128(rank, implicit, alpha):
    """BASELINE configs[2] in miniature: implicit alpha=40, rank 128, 5 iterations (the
    4-wave workgroup path), factors vs the fp64 oracle after every iteration."""
    u, i, r = planted(700, 450, density=0.05, seed=13, heavy_items=(4,), dup=20)
    core = _core(u, i, r, chunk=256)
    worst, *_ = _fit_per_iteration(core, u, i, r, rank, 5, 0.1, implicit, alpha)
    report(f"full_fit_per_iteration[rank={rank},implicit={implicit}]", worst)


@pytest.mark.parametrize("outlier,implicit", [(1e2, False), (1e4, False), (1e5, False),
                                              (1e2, True), (1e4, True)])
@pytest.mark.parametrize("rank", [16, 64, 128])
def test_half_sweep_mixed_row_norms(outlier, implicit, rank):
    """The split-f16 scale is one power of two per launch (from max |Y|): a block of
    users whose factors are `outlier` times larger (600 users, own items) must not cost the other rows
    their precision.  The outlier users rate a disjoint set of items, so every
    system stays well conditioned and only the shared scale is exercised
    (documented range, DESIGN.md §K2: entries down to ~1e-5 of the largest keep
    fp32-grade products; an ill-conditioned system is limited by the fp32
    factorisation instead, cond(A) x 6e-8)."""
    u1, i1, r1 = planted(760, 380, density=0.05, heavy_items=(3,), seed=23)
    # the outlier block: 600 users x 10 items, all rated, so its own systems are
    # well conditioned at every rank (cond ~ (1 + sqrt(k/600))^2 / (1 - sqrt(k/600))^2)
    u2, i2, r2 = planted(600, 10, density=1.0, seed=24)
    u = np.concatenate([u1, u2 + 760]).astype(np.int32)
    i = np.concatenate([i1, i2 + 380]).astype(np.int32)
    r = np.concatenate([r1, r2]).astype(np.float32)
    core = _core(u, i, r, chunk=256)
    core.init_factors(rank, seed=3)
    core.U[760:] *= outlier  # dense rows = ids here (ids 0..799 all present)
    U0 = core.U[:, :rank].cpu().numpy()
    alpha = 40.0 if implicit else 1.0  # implicit: the split-f16 W1 Schur at rank 128
    core.half_sweep_items(0.1, implicit, alpha)
    torch.cuda.synchronize()
    core.check_status()
    ib = core.item_block
    V_ref = O.half_sweep(ib.row_ptr.cpu().numpy(), ib.col.cpu().numpy(), ib.val.cpu().numpy(),
                         U0, 0.1, implicit, alpha)
    ev = rel_row_err(core.V[:, :rank].cpu().numpy(), V_ref)
    report(f"half_sweep_mixed_norms[x{outlier:g},rank={rank},implicit={implicit}]", ev)
    assert ev <= 1e-4


def _degree_data(degrees, n_items, seed):
    """Users with exactly the given degrees (distinct items each) plus one user rating
    every item (so every item is rated); planted half-star ratings."""
    rng = np.random.default_rng(seed)
    us = [np.full(d, uid) for uid, d in enumerate(degrees)]
    its = [rng.choice(n_items, d, replace=False) for d in degrees]
    us.append(np.full(n_items, len(degrees)))
    its.append(np.arange(n_items))
    u = np.concatenate(us).astype(np.int32)
    i = np.concatenate(its).astype(np.int32)
    uf = rng.normal(0, 0.35, (len(degrees) + 1, 8))
    vf = rng.normal(0, 0.35, (n_items, 8))
    r = np.clip(np.round((3.6 + (uf[u] * vf[i]).sum(1) + rng.normal(0, 0.8, len(u))) * 2) / 2,
                0.5, 5).astype(np.float32)
    return u, i, r


DUAL_DEGREES = [1, 2, 7, 15, 16, 17, 31, 32, 33, 40, 47, 48, 49, 63, 64, 65, 66, 90, 96, 97, 128, 129]


@pytest.mark.parametrize("rank,reg", [(33, 0.1), (40, 0.1), (48, 0.1), (64, 0.1), (64, 1e-3),
                                      (64, 1e-4), (65, 0.1), (96, 0.1),
                                      (100, 0.1), (128, 0.1), (65, 1e-3), (80, 1e-3), (95, 1e-3),
                                      (80, 1e-4), (128, 1e-3)])
def test_dual_short_rows_match_primal_and_oracle(rank, reg):
    """Explicit rows with <= min(96, rank) ratings at rank 65-128 go through the n x n
    dual system (NB = 2 for n <= 32, 4 for n <= 64, 6 for n <= 96), rows with <= 32
    ratings at rank 33-64 too (NB = 2, split table of 64 words per row); the rest
    through the k x k primal.  The limit min(96, rank) keeps the dual system full rank
    (n <= k): at rank 65-95 the rows with rank < n <= 96 stay primal, which the small
    regParams (1e-3, 1e-4) would otherwise expose.  Both forms vs the fp64 oracle of
    Spark's k x k normal equations, per row, with the degrees around every class
    boundary (1, 16/17, 32/33, 64/65, 96/97) and at the rank limit."""
    degrees = (DUAL_DEGREES + [rank - 1, rank, rank + 1]) * 15
    u, i, r = _degree_data(degrees, 400, seed=rank)
    core = _core(u, i, r, chunk=256)
    ub = core.user_block
    assert ub.n_short == sum(d <= E.DUAL_MAX_RATINGS for d in degrees)
    assert ub.n_dual(rank) == sum(d <= E.dual_limit(rank) for d in degrees)
    assert E.dual_limit(rank) == (min(96, rank) if rank > 64 else 32)
    core.init_factors(rank, seed=3)
    g = torch.Generator(device=DEV)
    g.manual_seed(rank)
    V0 = torch.randn((core.n_items, rank), generator=g, device=DEV)
    V0 = V0 / torch.linalg.vector_norm(V0, dim=1, keepdim=True)
    core.V[:, :rank] = V0
    V0 = V0.cpu().numpy()
    U_ref = O.half_sweep(ub.row_ptr.cpu().numpy(), ub.col.cpu().numpy(), ub.val.cpu().numpy(),
                         V0, reg)
    deg = np.diff(ub.row_ptr.cpu().numpy())
    out = {}
    for dual in (True, False):
        core.U.fill_(7.0)  # every written entry must be overwritten (pad columns with 0)
        core.status.zero_()
        E.solve_half(ub, core.V, core.U, rank, reg, False, 1.0, None, core.status, core.ws,
                     dual=dual)
        torch.cuda.synchronize()
        core.check_status()
        U = core.U.cpu().numpy()
        assert np.all(U[:, rank:] == 0.0)
        e = rel_row_errs(U[:, :rank], U_ref)
        out[dual] = {f"deg<={b}": float(e[(deg <= b) & (deg > a)].max())
                     for a, b in ((0, 16), (16, 32), (32, 48), (48, 64), (64, 10 ** 9))
                     if ((deg <= b) & (deg > a)).any()}
        assert e.max() <= 1e-4, (dual, out[dual])
    report(f"dual_vs_primal[rank={rank},reg={reg:g}]", out)


def test_dual_rows_in_any_order():
    """The dual kernel picks its block count per row (NB = 6 / 4 / 2 for 65-96, 33-64,
    <= 32 ratings), so the dual tail of the light list may come in any order: reversed
    and shuffled tails give the same rows as the longest-first one (round 4 measured
    three per-class launches over the sorted ranges: 70.4 vs 67.3 ms at configs[3] —
    the mixed launch overlaps the matrix-core-heavy long rows with the short ones)."""
    rank, reg = 128, 0.1
    degrees = DUAL_DEGREES * 20
    u, i, r = _degree_data(degrees, 400, seed=11)
    core = _core(u, i, r, chunk=256)
    ub = core.user_block
    core.init_factors(rank, seed=3)
    # unit-norm random item factors (init_factors leaves V at zero: the item side is
    # solved first), so every user row has a non-trivial solution to compare
    g = torch.Generator(device=DEV)
    g.manual_seed(17)
    V0 = torch.randn((core.n_items, rank), generator=g, device=DEV)
    V0 = V0 / torch.linalg.vector_norm(V0, dim=1, keepdim=True)
    core.V[:, :rank] = V0
    V0 = V0.cpu().numpy()
    U_ref = O.half_sweep(ub.row_ptr.cpu().numpy(), ub.col.cpu().numpy(), ub.val.cpu().numpy(),
                         V0, reg)
    assert np.linalg.norm(U_ref, axis=1).min() > 0
    nd = ub.n_dual(rank)
    assert nd > 0
    n_primal = ub.n_light - nd
    g = torch.Generator(device="cpu")
    g.manual_seed(5)
    for order in ("reversed", "shuffled"):
        tail = ub.light_rows[n_primal:ub.n_light].clone()
        tail = tail.flip(0) if order == "reversed" else tail[torch.randperm(nd, generator=g).to(DEV)]
        blk = dataclasses.replace(ub, light_rows=torch.cat([ub.light_rows[:n_primal], tail]))
        core.U.fill_(7.0)
        core.status.zero_()
        E.solve_half(blk, core.V, core.U, rank, reg, False, 1.0, None, core.status, core.ws)
        torch.cuda.synchronize()
        core.check_status()
        e = rel_row_errs(core.U[:, :rank].cpu().numpy(), U_ref)
        report(f"dual_unordered[{order}]", {"max_rel": float(e.max())})
        assert e.max() <= 1e-4, (order, float(e.max()))


def _exact_rel_errs(x, ref):
    """Per-row ||x - ref|| / ||ref|| with no floor (rows of any magnitude)."""
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    nr = np.linalg.norm(ref, axis=1)
    e = np.linalg.norm(x - ref, axis=1) / np.where(nr > 0, nr, 1.0)
    e[nr == 0] = np.linalg.norm(x[nr == 0], axis=1)
    return e


@pytest.mark.parametrize("spread", [1e7, 1e9])
@pytest.mark.parametrize("rank", [16, 48, 64, 100, 128])
def test_split_window_row_norm_spread(spread, rank):
    """Split window guard: the explicit Gram uses one power-of-two scale
    per launch, so factor rows far below the launch maximum would reach subnormal f16
    lo halves.  A block of users whose factors are 1/spread of the rest rates its own
    items (light rows, dual-path short rows and one heavy, chunked item): those items'
    systems see only tiny factor rows and must still match the fp64 oracle to 1e-4
    per row — relative to their own norm — via the rescue launch."""
    u1, i1, r1 = planted(500, 300, density=0.05, heavy_items=(3,), seed=31)
    u2, i2, r2 = planted(400, 120, density=0.08, heavy_items=(5,), seed=32)  # tiny users' items
    u = np.concatenate([u1, u2 + 500]).astype(np.int32)
    i = np.concatenate([i1, i2 + 300]).astype(np.int32)
    r = np.concatenate([r1, r2]).astype(np.float32)
    core = _core(u, i, r, chunk=128)
    core.init_factors(rank, seed=3)
    core.U[500:] /= spread
    U0 = core.U[:, :rank].cpu().numpy()
    core.half_sweep_items(0.1, False, 1.0)
    torch.cuda.synchronize()
    core.check_status()
    ib = core.item_block
    V_ref = O.half_sweep(ib.row_ptr.cpu().numpy(), ib.col.cpu().numpy(), ib.val.cpu().numpy(),
                         U0, 0.1)
    e = _exact_rel_errs(core.V[:, :rank].cpu().numpy(), V_ref)
    tiny = np.arange(300, 420)  # dense rows = ids (all present)
    report(f"split_window_norm_spread[{spread:g},rank={rank}]",
           {"tiny_rows": float(e[tiny].max()), "other_rows": float(np.delete(e, tiny).max())})
    assert e.max() <= 1e-4, (e[tiny].max(), np.delete(e, tiny).max())
    # and the reverse direction: the tiny items' factors feed a user half-sweep
    core.V[:, :rank] = torch.as_tensor(V_ref).to(DEV)
    core.half_sweep_users(0.1, False, 1.0)
    ub = core.user_block
    U_ref = O.half_sweep(ub.row_ptr.cpu().numpy(), ub.col.cpu().numpy(), ub.val.cpu().numpy(),
                         V_ref, 0.1)
    eu = _exact_rel_errs(core.U[:, :rank].cpu().numpy(), U_ref)
    assert eu.max() <= 1e-4


def test_rescue_list_emptied_between_row_chunks():
    """Row chunks of one half-sweep share one Y prep (the sharded engine's chunk calls run
    every phase but PREP): the rescue list a call fills must be empty again when the next
    call's LAUNCH1 starts (the rescue launch's last block clears it), or rows of one
    chunk would be re-solved with the next chunk's CSR.  Counted directly: the list
    length (scale word 2) after LAUNCH1..LAUNCH2 is the same in both calls, and 0 after
    RESCUE."""
    rank, spread = 64, 1e9
    u1, i1, r1 = planted(500, 300, density=0.05, heavy_items=(3,), seed=31)
    u2, i2, r2 = planted(400, 120, density=0.08, heavy_items=(5,), seed=32)
    u = np.concatenate([u1, u2 + 500]).astype(np.int32)
    i = np.concatenate([i1, i2 + 300]).astype(np.int32)
    r = np.concatenate([r1, r2]).astype(np.float32)
    core = _core(u, i, r, chunk=128)
    core.init_factors(rank, seed=3)
    core.U[500:] /= spread
    U0 = core.U[:, :rank].cpu().numpy()
    ib = core.item_block
    V_ref = O.half_sweep(ib.row_ptr.cpu().numpy(), ib.col.cpu().numpy(), ib.val.cpu().numpy(),
                         U0, 0.1)

    def count():
        torch.cuda.synchronize()
        return int(core.ws.buf[8:12].view(torch.int32).item())
    counts = []
    for phases in (E.PHASE_ALL, E.PHASE_ALL & ~E.PHASE_PREP):
        core.V.fill_(7.0)
        core.status.zero_()
        E.solve_half(ib, core.U, core.V, rank, 0.1, False, 1.0, None, core.status, core.ws,
                     phases & ~E.PHASE_RESCUE)
        counts.append(count())
        E.solve_half(ib, core.U, core.V, rank, 0.1, False, 1.0, None, core.status, core.ws,
                     E.PHASE_RESCUE)
        assert count() == 0
        core.check_status()
        e = _exact_rel_errs(core.V[:, :rank].cpu().numpy(), V_ref)
        assert e.max() <= 1e-4, (phases, float(e.max()))
    report("rescue_list_between_chunks", {"rescued_per_call": counts})
    assert counts[0] > 0 and counts[0] == counts[1], counts


@pytest.mark.parametrize("rank", [16, 64, 128])
def test_blocks_sharing_one_prep(rank):
    """Row chunks of one half-sweep (the sharded engine's per-chunk blocks) share one Y
    prep: the second call skips PREP and must find the split table where the first call
    left it although the blocks differ in rows and heavy-row chunks (the table sits at
    the workspace's end; round 5 briefly placed it after the per-call slot / rescue
    regions, which moved it between such calls)."""
    from als_mi355x.distributed import HipKernels
    u, i, r = planted(700, 260, density=0.06, heavy_items=(3, 4, 5), seed=71)
    K = HipKernels(DEV, chunk=64)
    n_u = int(u.max()) + 1
    V0 = torch.zeros((n_u, E.ld_for(rank)), device=DEV)
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    V0[:, :rank] = torch.randn((n_u, rank), generator=g, device=DEV)
    parts = []
    for lo, hi in ((0, 40), (40, 260)):  # 40 rows incl. the heavy items, then 220 rows
        sel = (i >= lo) & (i < hi)
        blk = K.build_block(_t(i[sel] - lo, torch.int32), _t(u[sel], torch.int32),
                            _t(r[sel], torch.float32), hi - lo, n_u)
        parts.append(blk)
    assert parts[0].n_chunks > 0 and parts[0].n_light + parts[0].n_heavy != \
        parts[1].n_light + parts[1].n_heavy
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    shared = [torch.full((b.n_rows, V0.shape[1]), 7.0, device=DEV) for b in parts]
    for c, blk in enumerate(parts):
        K.solve_half(blk, V0, shared[c], rank, 0.1, False, 1.0, None, st, first=(c == 0))
    alone = []
    for blk in parts:
        X = torch.full((blk.n_rows, V0.shape[1]), 7.0, device=DEV)
        E.solve_half(blk, V0, X, rank, 0.1, False, 1.0, None, st, E.Workspace(DEV))
        alone.append(X)
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    for a, b in zip(shared, alone):
        assert torch.equal(a, b)


@pytest.mark.parametrize("implicit", [False, True])
@pytest.mark.parametrize("rank", [8, 16, 48, 64, 100, 128])
def test_two_segment_half_sweep(rank, implicit):
    """ABI 6 two-segment schedule (the sharded engine's pipelined item side): every
    item row's ratings ordered early-first — users below a cut (the arrived prefix of
    Y), then the rest — the early call reads only that prefix (the rows past it hold NaN
    during the call, as a chunk still in flight would hold anything), the late call
    adds the remaining partials, sums every row's slots in fp64 and solves.  Against
    the one-call solve of the same block and the fp64 oracle; chunk 64 so long rows
    span several tasks of each segment, including the heavy item."""
    u, i, r = planted(600, 200, density=0.08, heavy_items=(3,), seed=61)
    if implicit:
        r = (r - 2.5).astype(np.float32)
    cut = 360  # users [0, cut) are the early prefix (dense user rows = ids here)
    late = u >= cut
    o = np.argsort(late, kind="stable")  # early ratings first in every row (stable CSR)
    core = _core(u[o], i[o], r[o], chunk=64)
    assert core.uidx.n == 600
    core.init_factors(rank, seed=7)
    ib = core.item_block
    rp = ib.row_ptr.cpu().numpy()
    col = ib.col.cpu().numpy()
    seg = rp[:-1] + np.add.reduceat((col < cut).astype(np.int64), rp[:-1]) * (np.diff(rp) > 0)
    assert (col[np.arange(len(col)) < np.repeat(seg, np.diff(rp))] < cut).all()
    sched = E.split_schedule(ib, _t(seg, torch.int64), cut, chunk=64)
    yty = E.compute_yty(core.U, core.n_users, rank, core.ws) if implicit else None
    alpha = 2.0
    # one-call reference on the same block
    core.status.zero_()
    E.solve_half(ib, core.U, core.V, rank, 0.1, implicit, alpha, yty, core.status, core.ws,
                 dual=False)
    V1 = core.V.clone()
    U0 = core.U[:, :rank].cpu().numpy()
    ws = E.Workspace(DEV)
    Vs = torch.full_like(core.V, 7.0)
    held = core.U[cut:].clone()
    core.U[cut:] = float("nan")
    E.solve_half_split(ib, sched, "early", core.U, Vs, rank, 0.1, implicit, alpha, yty,
                       core.status, ws)
    core.U[cut:] = held  # the last chunk "arrives" (stream order)
    E.solve_half_split(ib, sched, "late", core.U, Vs, rank, 0.1, implicit, alpha, yty,
                       core.status, ws)
    torch.cuda.synchronize()
    core.check_status()
    Vs_np = Vs[:, :rank].cpu().numpy()
    assert np.all(Vs[:, rank:].cpu().numpy() == 0.0)
    V_ref = O.half_sweep(rp, col, ib.val.cpu().numpy(), U0, 0.1, implicit, alpha)
    e_one = float(_exact_rel_errs(Vs_np, V1[:, :rank].cpu().numpy()).max())
    e_ref = float(_exact_rel_errs(Vs_np, V_ref).max())
    report(f"two_segment[rank={rank},imp={int(implicit)}]",
           {"vs_one_call": e_one, "vs_oracle": e_ref, "early_tasks": sched.early[3],
            "late_tasks": sched.late[3]})
    assert sched.early[3] > 0 and sched.late[3] > 0
    assert e_ref <= (1e-5 if implicit and rank <= 64 else 1e-4) and e_one <= 1e-4, (e_one, e_ref)


@pytest.mark.parametrize("rank", [16, 64, 128])
def test_rescue_list_overflow_is_an_error(rank):
    """A caller that runs the LAUNCH phases twice without RESCUE between them appends
    every flagged row twice: with most rows flagged that passes the list's capacity (the
    block's rows).  The kernels never write past it, and the RESCUE launch reports the
    overflow (status -1) instead of walking a list longer than its storage."""
    spread = 1e9
    u1, i1, r1 = planted(120, 20, density=0.3, seed=31)
    u2, i2, r2 = planted(400, 120, density=0.08, seed=32)  # tiny users' items: flagged
    u = np.concatenate([u1, u2 + 120]).astype(np.int32)
    i = np.concatenate([i1, i2 + 20]).astype(np.int32)
    r = np.concatenate([r1, r2]).astype(np.float32)
    core = _core(u, i, r, chunk=128)
    core.init_factors(rank, seed=3)
    core.U[120:] /= spread
    ib = core.item_block
    core.status.zero_()
    once = E.PHASE_ALL & ~E.PHASE_RESCUE
    E.solve_half(ib, core.U, core.V, rank, 0.1, False, 1.0, None, core.status, core.ws, once)
    torch.cuda.synchronize()
    n_flagged = int(core.ws.buf[8:12].view(torch.int32).item())
    assert 2 * n_flagged > ib.n_light + ib.n_heavy, n_flagged
    E.solve_half(ib, core.U, core.V, rank, 0.1, False, 1.0, None, core.status, core.ws,
                 once & ~E.PHASE_PREP)
    E.solve_half(ib, core.U, core.V, rank, 0.1, False, 1.0, None, core.status, core.ws,
                 E.PHASE_RESCUE)
    torch.cuda.synchronize()
    report(f"rescue_overflow[rank={rank}]", {"flagged": n_flagged,
                                             "rows": ib.n_light + ib.n_heavy})
    with pytest.raises(RuntimeError, match="rescue list overflow"):
        core.check_status()
    # the list was emptied by that RESCUE launch: a normal call is clean again
    core.status.zero_()
    core.half_sweep_items(0.1, False, 1.0)
    torch.cuda.synchronize()
    core.check_status()


@pytest.mark.parametrize("rank", [8, 64, 128])
def test_split_window_rating_spread(rank):
    """Ratings spanning nine decades: users whose ratings are all ~1e-9 of the block's
    largest rating (the rhs split's lo halves would be subnormal) are re-solved with
    their own scale; every row matches the oracle to 1e-4 of its own norm."""
    u, i, r = planted(600, 300, density=0.06, heavy_users=(2,), seed=41)
    rng = np.random.default_rng(5)
    scale = np.where(u % 3 == 0, 1e-9, np.where(u % 3 == 1, 1.0, 1e3)).astype(np.float64)
    r = (r * scale * rng.uniform(0.5, 1.5, r.size)).astype(np.float32)
    core = _core(u, i, r, chunk=128)
    core.init_factors(rank, seed=4)
    g = torch.Generator(device=DEV)
    g.manual_seed(9)
    V0 = torch.randn((core.n_items, rank), generator=g, device=DEV)
    core.V[:, :rank] = V0
    core.half_sweep_users(0.1, False, 1.0)
    torch.cuda.synchronize()
    core.check_status()
    ub = core.user_block
    U_ref = O.half_sweep(ub.row_ptr.cpu().numpy(), ub.col.cpu().numpy(), ub.val.cpu().numpy(),
                         V0.cpu().numpy(), 0.1)
    e = _exact_rel_errs(core.U[:, :rank].cpu().numpy(), U_ref)
    report(f"split_window_rating_spread[rank={rank}]", float(e.max()))
    assert e.max() <= 1e-4


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("rank", [8, 16, 32, 64, 128])
def test_implicit_counts_spanning_six_decades(rank, seed):
    """Implicit feedback with counts 1..1e6 (alpha 1): the confidence weights span six
    decades and the systems' condition numbers reach ~1e4-1e5, which the fp32-grade Gram
    and fp32 LDL^T alone turn into 1e-4..4e-3 errors (emulated).  At rank <= 64 every
    implicit row is iteratively refined against Spark's fp64 residual (rows that do not
    converge go to the fp64 rescue); at rank 65-128 the W1 solve's pivot-spread test
    routes rows whose pivots spread beyond 8 (kCondMaxImplicit) to the fp64 rescue.
    Every row (light rows and the chunked heavy item) must match the oracle to 2e-6 at
    ranks <= 64 (measured <= 7.1e-7) and 1e-6 at rank 128 (measured <= 8.4e-8; 5.6e-6
    with round 5's limit of 32) — 50-100x under the 1e-4 bar."""
    u, i, _ = planted(500, 300, density=0.06, heavy_items=(4,), seed=43 + 10 * seed)
    rng = np.random.default_rng(6 + seed)
    r = np.round(10.0 ** rng.uniform(0, 6, u.size)).astype(np.float32)
    core = _core(u, i, r, chunk=128)
    core.init_factors(rank, seed=5 + seed)
    U0 = core.U[:, :rank].cpu().numpy()
    core.half_sweep_items(0.1, True, 1.0)
    torch.cuda.synchronize()
    core.check_status()
    ib = core.item_block
    V_ref = O.half_sweep(ib.row_ptr.cpu().numpy(), ib.col.cpu().numpy(), ib.val.cpu().numpy(),
                         U0, 0.1, True, 1.0)
    e = _exact_rel_errs(core.V[:, :rank].cpu().numpy(), V_ref)
    report(f"implicit_counts_1_1e6[rank={rank},seed={seed}]", float(e.max()))
    assert e.max() <= (1e-6 if rank > 64 else 2e-6), float(e.max())


def test_failed_pivot_raises_with_row():
    """A singular system (Spark: dppsv info > 0) is reported, not silently solved:
    items rated only by users whose factors are zero, regParam 0 -> A = 0."""
    u, i, r = planted(200, 120, density=0.05, seed=4)
    core = _core(u, i, r)
    core.init_factors(8, seed=1)
    uid = core.uidx.map.cpu().numpy()
    # every user that rated item id 0 gets a zero factor row
    zero_users = np.unique(u[i == i.min()])
    U0 = core.U[:, :8].cpu().numpy()
    U0[uid[zero_users]] = 0.0
    with pytest.raises(RuntimeError, match="Cholesky failed"):
        core.fit(8, 1, 0.0, U0=U0)


# ---------------------------------------------------------------- K4
def test_predict_and_rmse_inner_join():
    u, i, r = planted(200, 150, density=0.1, seed=2, id_gap=2)
    core = _core(u, i, r)
    core.fit(10, 2, 0.1, seed=1)
    U = core.U[:, :10].cpu().numpy()
    V = core.V[:, :10].cpu().numpy()
    umap, imap = core.uidx.map.cpu().numpy(), core.iidx.map.cpu().numpy()
    rng = np.random.default_rng(0)
    pu = rng.integers(-3, int(u.max()) + 10, 5000).astype(np.int32)  # incl. unknown / odd ids
    pi = rng.integers(-3, int(i.max()) + 10, 5000).astype(np.int32)
    pr = rng.uniform(0.5, 5, 5000).astype(np.float32)
    got = core.predict(pu, pi).cpu().numpy()
    ref = O.predict(U, V, umap, imap, pu, pi)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert ok.sum() > 100
    np.testing.assert_allclose(got[ok], ref[ok], rtol=1e-9, atol=1e-12)
    rm, n = core.rmse(pu, pi, pr)
    sse, n_ref = O.rmse(U, V, umap, imap, pu, pi, pr)
    assert n == n_ref and abs(rm - math.sqrt(sse / n_ref)) <= 1e-9


def test_compute_error_kat_on_gpu():
    """output.txt:16-18 known answers through the fused RMSE kernel.

    Predicted ratings are injected as rank-1 factors: U[u] = pred, V[i] = 1
    would make every (u, i) the same; instead use rank = n_items one-hot item
    factors so <U[u], V[i]> = pred(u, i) exactly."""
    kat = json.load(open(os.path.join(HERE, "golden", "compute_error_kat.json")))
    for case in kat["cases"]:
        pred = case["predicted"]
        act = case["actual"]
        users = sorted({p[0] for p in pred} | {a[0] for a in act})
        items = sorted({p[1] for p in pred} | {a[1] for a in act})
        k = 4 * ((len(items) + 3) // 4)
        U = np.zeros((max(users) + 1, k), np.float32)
        V = np.zeros((max(items) + 1, k), np.float32)
        for j, it in enumerate(items):
            V[it, j] = 1.0
        known_u = np.full(max(users) + 1, -1, np.int32)
        known_i = np.full(max(items) + 1, -1, np.int32)
        for uu, ii, pp in pred:
            U[uu, items.index(ii)] = pp
            known_u[uu] = uu
            known_i[ii] = ii
        uidx = E.IdIndex(_t(known_u, torch.int32), _t(np.unique(known_u[known_u >= 0]),
                                                     torch.int32), 0)
        # pairs whose (u, i) is not in `pred` must drop out: encode by per-pair filtering
        pset = {(p[0], p[1]) for p in pred}
        act_in = [a for a in act if (a[0], a[1]) in pset]
        a = np.array(act_in, dtype=np.float64).reshape(-1, 3)
        iidx = E.IdIndex(_t(known_i, torch.int32), _t(np.unique(known_i[known_i >= 0]),
                                                     torch.int32), 0)
        out = E.rmse_pairs(_t(a[:, 0], torch.int32), _t(a[:, 1], torch.int32),
                           _t(a[:, 2], torch.float32), uidx, iidx, _t(U, torch.float32),
                           _t(V, torch.float32), k, E.Workspace(DEV)).cpu().numpy()
        got = math.sqrt(out[0] / out[1])
        assert round(got, 11) == pytest.approx(case["expected"], abs=1e-11)


# ---------------------------------------------------------------- K5
@pytest.mark.parametrize("rank,top", [(4, 1), (10, 10), (32, 20), (64, 8), (64, 9), (64, 10), (64, 12), (64, 13), (64, 16), (16, 17), (64, 100),
                                      (64, 256), (96, 10), (128, 100), (128, 253),
                                      # quad register lists (16 < top <= 128) at their size boundaries
                                      (64, 32), (64, 33), (128, 64), (32, 65), (64, 99), (128, 101), (128, 128),
                                      (128, 129)])
def test_topk_parity(rank, top):
    rng = np.random.default_rng(rank * 1000 + top)
    n_q, n_v = 333, 1500
    Q = rng.standard_normal((n_q, rank)).astype(np.float32)
    Vm = rng.standard_normal((n_v, rank)).astype(np.float32)
    Vm[10] = Vm[20]  # exact tie: the lower index must come first
    ld = E.ld_for(rank)
    Qd = torch.zeros((n_q, ld), device=DEV)
    Qd[:, :rank] = torch.as_tensor(Q).to(DEV)
    Vd = torch.zeros((n_v, ld), device=DEV)
    Vd[:, :rank] = torch.as_tensor(Vm).to(DEV)
    idx, sc = E.topk_rows(Qd, n_q, Vd, n_v, rank, top)
    idx, sc = idx.cpu().numpy(), sc.cpu().numpy()
    ref_i, ref_s = O.topk(Q, Vm, top)
    S = Q.astype(np.float64) @ Vm.astype(np.float64).T
    for row in range(n_q):
        if not np.array_equal(idx[row], ref_i[row]):
            # only tolerated where fp64 scores tie within 1e-5
            bad = np.nonzero(idx[row] != ref_i[row])[0]
            for p in bad:
                assert abs(S[row, idx[row, p]] - ref_s[row, p]) <= 1e-5 * max(1, abs(ref_s[row, p]))
        np.testing.assert_allclose(sc[row], ref_s[row], rtol=1e-5, atol=1e-5)
    both = [r_ for r_ in range(n_q) if 10 in ref_i[r_] and 20 in ref_i[r_]]
    for r_ in both:
        lst = list(idx[r_])
        assert lst.index(10) < lst.index(20)


@pytest.mark.parametrize("rank,n_v,top", [(64, 20011, 10), (128, 9001, 10), (32, 17, 10),
                                          (16, 300, 10), (128, 9001, 100), (64, 20011, 50)])
def test_topk_many_tiles_ties_across_tiles(rank, n_v, top):
    """Many V tiles, a ragged last tile, and exact ties whose copies sit in different
    tiles and blocks (the lower index must win wherever the copies fall)."""
    rng = np.random.default_rng(rank + n_v + top)
    n_q = 261
    Q = rng.standard_normal((n_q, rank)).astype(np.float32)
    Vm = rng.standard_normal((n_v, rank)).astype(np.float32)
    Vm *= (1.0 + 3.0 * (np.arange(n_v) % 97 == 0))[:, None].astype(np.float32)  # strong items
    pairs = [(a, b) for a, b in ((0, n_v - 1), (5, 4100), (130, 131), (97, 8999)) if b < n_v]
    for a, b in pairs:
        Vm[b] = Vm[a]
    ld = E.ld_for(rank)
    Qd = torch.zeros((n_q, ld), device=DEV)
    Qd[:, :rank] = torch.as_tensor(Q).to(DEV)
    Vd = torch.zeros((n_v, ld), device=DEV)
    Vd[:, :rank] = torch.as_tensor(Vm).to(DEV)
    idx, sc = E.topk_rows(Qd, n_q, Vd, n_v, rank, top)
    idx, sc = idx.cpu().numpy(), sc.cpu().numpy()
    ref_i, ref_s = O.topk(Q, Vm, top)
    S = Q.astype(np.float64) @ Vm.astype(np.float64).T
    for row in range(n_q):
        if not np.array_equal(idx[row], ref_i[row]):
            bad = np.nonzero(idx[row] != ref_i[row])[0]
            for p_ in bad:
                assert abs(S[row, idx[row, p_]] - ref_s[row, p_]) <= 1e-5 * max(1, abs(ref_s[row, p_]))
        np.testing.assert_allclose(sc[row], ref_s[row], rtol=1e-5, atol=1e-5)
        lst = list(idx[row])
        for a, b in pairs:
            if a in lst and b in lst:
                assert lst.index(a) < lst.index(b)
    assert any(a in idx[r_] and b in idx[r_] for r_ in range(n_q) for a, b in pairs)


@pytest.mark.parametrize("rank,top", [(64, 10), (128, 10), (32, 40), (128, 100)])
def test_topk_zero_rows_and_norm_order_ties(rank, top):
    """The sweep visits V by decreasing norm: ties between equal rows far apart in index
    (the large-norm copy visited first) must still resolve to the lower index; all-zero
    query rows list the first `top` items with score 0; zero V rows score 0."""
    rng = np.random.default_rng(rank + top)
    n_q, n_v = 300, 5000
    Q = rng.standard_normal((n_q, rank)).astype(np.float32)
    Q[[0, 7, 299]] = 0.0
    Vm = (rng.standard_normal((n_v, rank)) * rng.uniform(0.1, 3.0, (n_v, 1))).astype(np.float32)
    Vm[100:140] = 0.0
    big = np.argsort(-np.linalg.norm(Vm, axis=1))[:30]  # strong rows, copied to lower indices
    low = [t for t in range(100) if t not in set(big.tolist())][:30]  # copies never overwrite a source
    for t, b in zip(low, big):
        Vm[t] = Vm[b]
    ld = E.ld_for(rank)
    Qd = torch.zeros((n_q, ld), device=DEV)
    Qd[:, :rank] = torch.as_tensor(Q).to(DEV)
    Vd = torch.zeros((n_v, ld), device=DEV)
    Vd[:, :rank] = torch.as_tensor(Vm).to(DEV)
    idx, sc = E.topk_rows(Qd, n_q, Vd, n_v, rank, top)
    idx, sc = idx.cpu().numpy(), sc.cpu().numpy()
    ref_i, ref_s = O.topk(Q, Vm, top)
    S = Q.astype(np.float64) @ Vm.astype(np.float64).T
    for row in range(n_q):
        if not np.array_equal(idx[row], ref_i[row]):
            bad = np.nonzero(idx[row] != ref_i[row])[0]
            for p_ in bad:
                assert abs(S[row, idx[row, p_]] - ref_s[row, p_]) <= 1e-5 * max(1, abs(ref_s[row, p_]))
        np.testing.assert_allclose(sc[row], ref_s[row], rtol=1e-5, atol=1e-5)
        lst = list(idx[row])
        for t, b in zip(low, big):  # exact copies: the lower index first
            if t in lst and b in lst:
                assert lst.index(t) < lst.index(b)
    for row in (0, 7, 299):
        assert list(idx[row]) == list(range(top)) and np.all(sc[row] == 0)


@pytest.mark.parametrize("rank,top", [(32, 20), (64, 100), (128, 100), (128, 128)])
def test_topk_log_overflow_exact_ties(rank, top):
    """16 < top <= 128 keeps each row's keys in a log (csrc/topk.hip kTkLogCap keys): every
    key reaching the row's threshold is appended, ties included.  3,000 exact copies of
    one strong V row tie for every query that scores it
    high: in every row that lists a copy, all 3,000 copies reach the running k-th score
    and the log, which overflows and is cut to the row's `top` best keys mid-sweep (the
    index decides among the copies), several times: the listed copies must be exactly
    the lowest-index ones, in index order, after every better-scoring row."""
    rng = np.random.default_rng(rank + top + 11)
    n_q, n_v, n_copy = 200, 6000, 3000
    Q = rng.standard_normal((n_q, rank)).astype(np.float32)
    Vm = rng.standard_normal((n_v, rank)).astype(np.float32)
    copies = np.sort(rng.choice(n_v, n_copy, replace=False))
    Vm[copies] = 3.0 * Vm[copies[0]]  # one strong row, 3,000 times
    ld = E.ld_for(rank)
    Qd = torch.zeros((n_q, ld), device=DEV)
    Qd[:, :rank] = torch.as_tensor(Q).to(DEV)
    Vd = torch.zeros((n_v, ld), device=DEV)
    Vd[:, :rank] = torch.as_tensor(Vm).to(DEV)
    idx, sc = E.topk_rows(Qd, n_q, Vd, n_v, rank, top)
    idx, sc = idx.cpu().numpy(), sc.cpu().numpy()
    ref_i, ref_s = O.topk(Q, Vm, top)
    S = Q.astype(np.float64) @ Vm.astype(np.float64).T
    is_copy = np.zeros(n_v, bool)
    is_copy[copies] = True
    with_copies = 0
    for row in range(n_q):
        got = idx[row]
        listed = got[is_copy[got]]
        # the copies listed are the lowest-index ones, in index order
        np.testing.assert_array_equal(listed, copies[:len(listed)])
        np.testing.assert_array_equal(listed, ref_i[row][is_copy[ref_i[row]]])
        if not np.array_equal(got, ref_i[row]):
            for p_ in np.nonzero(got != ref_i[row])[0]:
                assert abs(S[row, got[p_]] - ref_s[row, p_]) <= 1e-5 * max(1, abs(ref_s[row, p_]))
        np.testing.assert_allclose(sc[row], ref_s[row], rtol=1e-5, atol=1e-5)
        # a listed copy scores >= the row's k-th: all 3,000 copies reached the log
        with_copies += len(listed) > 0
    assert with_copies > 20


@pytest.mark.parametrize("rank,top", [(32, 20), (128, 100), (64, 200)])
def test_topk_large_v_lds_lists(rank, top):
    """More than 2^18 V rows (many tall quad-list tiles, a ragged last one), as at configs[4]."""
    rng = np.random.default_rng(rank + top + 7)
    n_q, n_v = 96, (1 << 18) + 1000
    Q = rng.standard_normal((n_q, rank)).astype(np.float32)
    Vm = rng.standard_normal((n_v, rank)).astype(np.float32)
    Vm[123456] = Vm[7]  # exact tie across the sweep: the lower index first
    ld = E.ld_for(rank)
    Qd = torch.zeros((n_q, ld), device=DEV)
    Qd[:, :rank] = torch.as_tensor(Q).to(DEV)
    Vd = torch.zeros((n_v, ld), device=DEV)
    Vd[:, :rank] = torch.as_tensor(Vm).to(DEV)
    idx, sc = E.topk_rows(Qd, n_q, Vd, n_v, rank, top)
    idx, sc = idx.cpu().numpy(), sc.cpu().numpy()
    ref_i, ref_s = O.topk(Q, Vm, top)
    S = Q.astype(np.float64) @ Vm.astype(np.float64).T
    for row in range(n_q):
        if not np.array_equal(idx[row], ref_i[row]):
            bad = np.nonzero(idx[row] != ref_i[row])[0]
            for p_ in bad:
                assert abs(S[row, idx[row, p_]] - ref_s[row, p_]) <= 1e-5 * max(1, abs(ref_s[row, p_]))
        np.testing.assert_allclose(sc[row], ref_s[row], rtol=1e-5, atol=1e-5)
        lst = list(idx[row])
        if 7 in lst and 123456 in lst:
            assert lst.index(7) < lst.index(123456)


@pytest.mark.parametrize("n_v,top", [(5, 12), (5, 40), (37, 100), (70, 128)])
def test_topk_fewer_items_than_top(n_v, top):
    """Lists that never fill: the real entries in score order, then -1 / -inf."""
    Q = torch.randn(70, 8, device=DEV)
    Vm = torch.randn(n_v, 8, device=DEV)
    idx, sc = E.topk_rows(Q, 70, Vm, n_v, 8, top)
    idx, sc = idx.cpu().numpy(), sc.cpu().numpy()
    assert np.all(idx[:, n_v:] == -1) and np.all(sc[:, n_v:] == -np.inf)
    assert np.all(np.sort(idx[:, :n_v], axis=1) == np.arange(n_v))
    ref_i, ref_s = O.topk(Q.cpu().numpy(), Vm.cpu().numpy(), n_v)
    np.testing.assert_allclose(sc[:, :n_v], ref_s, rtol=1e-5, atol=1e-5)


def _topk_check(Q, Vm, idx, sc, top, tol=1e-5):
    """idx/sc vs the fp64 oracle: identical except where fp64 scores tie within tol."""
    ref_i, ref_s = O.topk(Q, Vm, top)
    S = Q.astype(np.float64) @ Vm.astype(np.float64).T
    for row in range(Q.shape[0]):
        if not np.array_equal(idx[row], ref_i[row]):
            bad = np.nonzero(idx[row] != ref_i[row])[0]
            for p_ in bad:
                assert abs(S[row, idx[row, p_]] - ref_s[row, p_]) <= tol * max(1, abs(ref_s[row, p_])), \
                    (row, p_, idx[row, p_], ref_i[row, p_])
        np.testing.assert_allclose(sc[row], ref_s[row], rtol=1e-5, atol=1e-5)
    return ref_i, ref_s


def _topk_dev(Q, Vm, rank, top):
    ld = E.ld_for(rank)
    Qd = torch.zeros((Q.shape[0], ld), device=DEV)
    Qd[:, :rank] = torch.as_tensor(Q).to(DEV)
    Vd = torch.zeros((Vm.shape[0], ld), device=DEV)
    Vd[:, :rank] = torch.as_tensor(Vm).to(DEV)
    idx, sc = E.topk_rows(Qd, Q.shape[0], Vd, Vm.shape[0], rank, top)
    return idx.cpu().numpy(), sc.cpu().numpy()


@pytest.mark.parametrize("rank,top", [(64, 10), (128, 10), (128, 100), (32, 40), (128, 200)])
def test_topk_scores_finer_than_f16(rank, top):
    """The coarse filter scores hi.hi only (f16 rounding ~5e-4 relative): V rows that
    differ from one strong row by relative steps of 4e-5 (below the f16 resolution of
    every element, above the 1e-5 tie tolerance) must still be ranked by their exact
    fp32-grade scores, i.e. the refinement decides every near-threshold pair."""
    rng = np.random.default_rng(rank * 7 + top)
    n_q, n_v = 128, 6000
    Q = rng.standard_normal((n_q, rank)).astype(np.float32)
    Vm = rng.standard_normal((n_v, rank)).astype(np.float32)
    base = rng.standard_normal(rank).astype(np.float32) * 3.0
    fam = rng.permutation(n_v)[:400]  # a family of near-copies scattered over the index range
    steps = (1.0 + 4e-5 * rng.integers(-60, 60, fam.size)).astype(np.float32)
    Vm[fam] = base[None, :] * steps[:, None]
    Q[: n_q // 2] = np.abs(Q[: n_q // 2]) * np.sign(base)[None, :]  # half the rows favour the family
    idx, sc = _topk_dev(Q, Vm, rank, top)
    ref_i, _ = _topk_check(Q, Vm, idx, sc, top)
    assert np.isin(ref_i[: n_q // 2], fam).mean() > 0.5  # the family dominates those lists


@pytest.mark.parametrize("rank,top", [(64, 10), (128, 16), (128, 100), (64, 150)])
def test_topk_wide_norm_spread_early_exit(rank, top):
    """V norms spread over six decades (most rows tiny): the norm-ordered sweep lets a
    workgroup stop once no remaining row can reach its rows' k-th scores; query rows of
    very different norms share a wavefront; results must equal the full sweep's."""
    rng = np.random.default_rng(rank + 3 * top)
    n_q, n_v = 200, 40000
    Q = (rng.standard_normal((n_q, rank)) * 10.0 ** rng.uniform(-3, 3, (n_q, 1))).astype(np.float32)
    Vm = (rng.standard_normal((n_v, rank)) * 10.0 ** rng.uniform(-6, 0, (n_v, 1))).astype(np.float32)
    Vm[rng.permutation(n_v)[:300]] *= 50.0  # a few strong rows
    Q[17] = 0.0
    idx, sc = _topk_dev(Q, Vm, rank, top)
    _topk_check(Q, Vm, idx, sc, top)
    assert list(idx[17]) == list(range(top))


@pytest.mark.parametrize("rank,top", [(64, 10), (128, 100), (64, 200)])
def test_topk_nan_factor_row(rank, top):
    """A V row holding a NaN (e.g. a loaded model) scores NaN: it is never listed, and
    every other row ranks as if it were absent."""
    rng = np.random.default_rng(rank + top + 11)
    n_q, n_v = 150, 3000
    Q = rng.standard_normal((n_q, rank)).astype(np.float32)
    Vm = rng.standard_normal((n_v, rank)).astype(np.float32)
    Vm *= rng.uniform(0.2, 2.0, (n_v, 1)).astype(np.float32)
    bad = [5, 1234]
    Vm[5, 3] = np.nan
    Vm[1234, 0] = np.nan
    idx, sc = _topk_dev(Q, Vm, rank, top)
    assert not np.isin(idx, bad).any()
    keep = np.setdiff1d(np.arange(n_v), bad)
    ref_i, ref_s = O.topk(Q, Vm[keep], top)
    ref_i = keep[ref_i]
    S = Q.astype(np.float64) @ Vm[keep].astype(np.float64).T
    for row in range(n_q):
        if not np.array_equal(idx[row], ref_i[row]):
            for p_ in np.nonzero(idx[row] != ref_i[row])[0]:
                assert abs(Q[row].astype(np.float64) @ Vm[idx[row, p_]].astype(np.float64)
                           - ref_s[row, p_]) <= 1e-5 * max(1, abs(ref_s[row, p_]))
        np.testing.assert_allclose(sc[row], ref_s[row], rtol=1e-5, atol=1e-5)
    del S


@pytest.mark.parametrize("rank,implicit,fixed", [(64, False, None), (128, False, None),
                                                 (128, True, None), (128, False, 1024)])
def test_task_length_follows_the_fit(rank, implicit, fixed):
    """ALSCore(chunk=None) schedules each half-sweep with engine.chunk_for(rank, implicit)
    (16384 explicit at rank > 64, else 4096); an explicit chunk stays fixed.  The factors
    are the same fp64-checked solve either way: one item half-sweep against the oracle."""
    from oracle import c_oracle as C
    u, i, r = planted(300, 40, density=0.9, seed=21, heavy_items=(0, 1))
    core = E.ALSCore(u, i, r, device=DEV, chunk=fixed)
    core.init_factors(rank, seed=2)
    U0 = core.U[:, :rank].cpu().numpy()
    core.half_sweep_items(0.1, implicit=implicit, alpha=3.0)
    torch.cuda.synchronize()
    core.check_status()
    want = fixed if fixed is not None else E.chunk_for(rank, implicit)
    assert core.item_block.chunk == want and core.user_block.chunk == want
    b = core.item_block
    ref, st = C.half_sweep(b.row_ptr.cpu().numpy(), b.col.cpu().numpy(), b.val.cpu().numpy(), U0,
                           0.1, implicit=implicit, alpha=3.0)
    assert not st.any()
    err = rel_row_err(core.V[:, :rank].cpu().numpy(), ref)
    report(f"task_length[rank={rank},imp={int(implicit)},chunk={want}]", err)
    assert err < 1e-5, err
