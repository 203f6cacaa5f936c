"""The sharded engine at the scale it targets: BASELINE configs[3] (1e9 ratings,
10M users x 1M items, rank 128, explicit, regParam 0.1) through ShardedALS over a
1-rank RCCL ("nccl") group, with the chunking and the capped all_to_all rounds
bench.py's configs3 uses (auto chunks; every collective <= MAX_COLLECTIVE_BYTES).

The round-2 fault happened exactly here (an uncapped 4.0e9-byte routing call), and
round 3 only timed this path.  Here the sharded engine and the single-GPU engine are
built from the same device-generated ratings, start from the same seeded U (the
global draw both use), run one full ALS iteration each, and every row of U and V is
compared: the per-row arithmetic is the same kernels on the same ratings in the same
order, so the only difference allowed is the per-chunk rating scale of the split rhs
(each chunk block has its own max |rating|) — bar 1e-6 relative per row.

Reference: RecommenderSystem.py:148-149 (ALS.train), SURVEY §8(e)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

import als_mi355x.datasets as D
import als_mi355x.engine as E
from helpers import report

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
RANK = 128
REG = 0.1


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _max_row_rel(a: torch.Tensor, b: torch.Tensor) -> float:
    """max over rows of ||a - b|| / ||b|| (rows of b that are zero: ||a||), on the GPU."""
    out = 0.0
    for s in range(0, a.shape[0], 1 << 20):
        x, y = a[s:s + (1 << 20)].double(), b[s:s + (1 << 20)].double()
        nd = torch.linalg.vector_norm(x - y, dim=1)
        ny = torch.linalg.vector_norm(y, dim=1)
        e = torch.where(ny > 0, nd / ny.clamp(min=1e-300), nd)
        out = max(out, float(e.max()))
    return out


def test_configs3_sharded_one_rank_matches_engine(monkeypatch):
    from als_mi355x import distributed as Dm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    calls = {"all_to_all_single": [0, 0], "all_gather_into_tensor": [0, 0]}

    def counted(name):
        fn = getattr(dist, name)

        def wrap(out, inp, *a, **kw):
            nb = max(out.numel() * out.element_size(), inp.numel() * inp.element_size())
            calls[name][0] += 1
            calls[name][1] = max(calls[name][1], nb)
            return fn(out, inp, *a, **kw)
        return wrap
    for name in calls:
        monkeypatch.setattr(Dm.dist, name, counted(name))
    try:
        u, i, r = D.big_config("big1b", device=DEV)
        # both engines pick the fit's task length (engine.chunk_for: 16384 ratings for
        # explicit rank 128): the same per-row arithmetic on both sides
        core = E.ALSCore(u, i, r, device=DEV)
        sh = Dm.ShardedALS(u, i, r, device=DEV)  # auto chunks, as bench.py configs3
        del u, i, r
        torch.cuda.empty_cache()
        assert core.nnz == sh.nnz == 1_000_000_000
        assert sh.users.chunks >= 2  # the chunked layout bench.py times
        # routing ran in capped rounds: 1e9 int32 = 4e9 B > 1 GiB per call otherwise
        assert calls["all_to_all_single"][0] > 2 * 3
        for name, (n, mx) in calls.items():
            assert mx <= Dm.MAX_COLLECTIVE_BYTES, (name, mx)
        core.init_factors(RANK, seed=5)
        sh.init_factors(RANK, seed=5)
        _, Us0 = sh.user_factors(cache=False)
        assert torch.equal(Us0, core.U[:, :RANK])  # the same global seeded draw
        del Us0
        core.status.zero_()
        sh.status.zero_()
        core.iterate(REG)
        sh.iterate(REG)
        torch.cuda.synchronize()
        core.check_status()
        sh.check_status()
        _, Vs = sh.item_factors(cache=False)
        ev = _max_row_rel(Vs, core.V[:, :RANK])
        del Vs
        _, Us = sh.user_factors(cache=False)
        eu = _max_row_rel(Us, core.U[:, :RANK])
        del Us
        for name, (n, mx) in calls.items():
            assert mx <= Dm.MAX_COLLECTIVE_BYTES, (name, mx)
        report("configs3_sharded_vs_engine_one_iteration",
               {"V_max_row_rel": ev, "U_max_row_rel": eu, "chunks": sh.users.chunks,
                "collectives": calls, "exchange": sh.exchange_stats(RANK)})
        assert all(b.chunk == E.chunk_for(RANK, False) for b in sh.user_blocks + sh.item_blocks
                   if b is not None)
        assert ev <= 1e-6 and eu <= 1e-6, (ev, eu)
    finally:
        dist.destroy_process_group()
