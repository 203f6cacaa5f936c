"""ShardedALS on the real HIP kernels with a 1-rank RCCL ("nccl") group: the
distributed code path (routing, padded layout, all_gather) must reproduce the
single-GPU engine from the same initial factors."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from helpers import planted, rel_row_err

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("implicit,chunks", [(False, None), (True, None), (False, 3)])
def test_sharded_one_rank_matches_engine(implicit, chunks):
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
        core.init_factors(16, seed=3)
        U0 = core.U[:, :16].cpu().numpy()
        core.fit(16, 3, 0.1, implicit=implicit, alpha=3.0, U0=U0)
        # chunks=3: the chunked [C, world, rows] layout with async per-chunk all-gathers
        sh = ShardedALS(u, i, r, device="cuda:0", chunks=chunks)
        sh.fit(16, 3, 0.1, implicit=implicit, alpha=3.0, U0_global=U0)
        _, Us = sh.user_factors()
        _, Vs = sh.item_factors()
        assert rel_row_err(Us.cpu().numpy(), core.U[:, :16].cpu().numpy()) < 1e-5
        assert rel_row_err(Vs.cpu().numpy(), core.V[:, :16].cpu().numpy()) < 1e-5
    finally:
        dist.destroy_process_group()
