"""ShardedALS on the real HIP kernels with a 1-rank RCCL ("nccl") group: the
distributed code path (routing, padded layout, all_gather) must reproduce the
single-GPU engine from the same initial factors."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from helpers import planted, rel_row_err, report

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("implicit,chunks,pipeline,rank",
                         [(False, None, None, 16), (True, None, None, 16), (False, 3, None, 16),
                          (False, 3, True, 16), (True, 3, True, 16), (False, 3, True, 64),
                          (True, 3, True, 64), (False, 3, True, 100), (True, 3, True, 128)])
def test_sharded_one_rank_matches_engine(implicit, chunks, pipeline, rank):
    """pipeline=True forces the pipelined item half-sweep at one rank (two-segment
    schedules: early partials from U chunks 0..C-2, late ones after the last chunk's
    all-gather, every row summed in fp64 and solved) — fp32 partials in another order,
    so 1e-5 against the single-GPU engine rather than bit-identity."""
    import als_mi355x.engine as E
    from als_mi355x.distributed import ShardedALS
    u, i, r = planted(400, 300, density=0.05, seed=7, heavy_items=(1,))
    if implicit:
        r = (r - 2.5).astype(np.float32)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        core = E.ALSCore(u, i, r, device="cuda:0", chunk=64)
        core.init_factors(rank, seed=3)
        U0 = core.U[:, :rank].cpu().numpy()
        core.fit(rank, 3, 0.1, implicit=implicit, alpha=3.0, U0=U0)
        # chunks=3: the chunked [C, world, rows] layout with async per-chunk all-gathers
        sh = ShardedALS(u, i, r, device="cuda:0", chunks=chunks, pipeline=pipeline)
        sh.fit(rank, 3, 0.1, implicit=implicit, alpha=3.0, U0_global=U0)
        assert sh.pipeline == bool(pipeline)
        _, Us = sh.user_factors()
        _, Vs = sh.item_factors()
        eu = rel_row_err(Us.cpu().numpy(), core.U[:, :rank].cpu().numpy())
        ev = rel_row_err(Vs.cpu().numpy(), core.V[:, :rank].cpu().numpy())
        report(f"sharded_one_rank[imp={int(implicit)},chunks={chunks},pipe={pipeline},"
               f"rank={rank}]", {"U": eu, "V": ev})
        assert eu < 1e-5 and ev < 1e-5, (eu, ev)
    finally:
        dist.destroy_process_group()
