"""One-process-per-GPU sharded ALS over torch.distributed (RCCL on ROCm).

Replaces Spark's data movement on the ALS path (SURVEY.md §2 "Spark
data-movement site" table, §8e):
  * partitionRatings / makeBlocks shuffles   -> one-time all_to_all(v) that routes
    every rating to the rank owning its user row and to the rank owning its
    item row;
  * computeFactors' srcOut.groupByKey        -> one all_gather of the updated factor
    half after each half-sweep (factors are replicated; each rank solves only
    its own rows);
  * computeYtY's treeAggregate (implicit)    -> local YtY of the rank's own rows +
    all_reduce of the k_pad^2 fp64 Gram.

Rows are split into contiguous, nnz-balanced ranges of the global dense index
(no row is split across ranks).  Every factor matrix lives in a *padded*
global layout [world, rows_per_rank, ld]: row `d` of owner `o` sits at
`o * rows_per_rank + (d - start[o])`, so the all-gathered buffer is directly
the gather table of the next half-sweep (no unpacking copy), and CSR column
indices are stored in that padded numbering.

The arithmetic is delegated to a `kernels` object (default: the HIP kernels of
libals_hip.so).  Tests substitute the CPU oracle to check the coordination
logic with the gloo backend on CPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist


class HipKernels:
    """The product kernels (libals_hip.so) behind the interface ShardedALS uses."""

    def __init__(self, device, chunk: Optional[int] = None):
        from . import engine as E
        self.E = E
        self.device = torch.device(device)
        self.ws = E.Workspace(self.device)
        self.chunk = chunk or E.DEFAULT_CHUNK

    def index_build(self, ids: torch.Tensor, id_space: int):
        idx = self.E.build_index(ids.to(self.device, torch.int32).contiguous(), id_space, self.ws)
        return idx.map, idx.uniq, idx.n

    def build_block(self, rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor,
                    n_rows: int, n_cols: int):
        ident_r = torch.arange(max(n_rows, 1), dtype=torch.int32, device=self.device)
        ident_c = torch.arange(max(n_cols, 1), dtype=torch.int32, device=self.device)
        ri = self.E.IdIndex(ident_r, ident_r, n_rows)
        ci = self.E.IdIndex(ident_c, ident_c, n_cols)
        return self.E.build_block(rows.contiguous(), ri, cols.contiguous(), ci,
                                  vals.contiguous(), self.ws, self.chunk)

    def yty(self, Y: torch.Tensor, n: int, rank: int) -> torch.Tensor:
        return self.E.compute_yty(Y, n, rank, self.ws)

    def solve_half(self, block, Y, X, rank, reg, implicit, alpha, yty, status):
        self.E.solve_half(block, Y, X, rank, reg, implicit, alpha, yty, status, self.ws)

    def ld(self, rank: int) -> int:
        return self.E.ld_for(rank)


def _all_gather_cat(t: torch.Tensor, world: int, group) -> torch.Tensor:
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return torch.cat(out)


def _ranges(deg: torch.Tensor, world: int):
    """Contiguous nnz-balanced row ranges: start[w] .. start[w+1]."""
    n = deg.numel()
    cum = torch.cumsum(deg.to(torch.float64), 0)
    total = float(cum[-1]) if n else 0.0
    targets = torch.tensor([total * w / world for w in range(1, world)], dtype=torch.float64,
                           device=deg.device)
    cut = torch.searchsorted(cum, targets, right=True) if n else torch.zeros(world - 1)
    starts = torch.cat([torch.zeros(1, device=deg.device, dtype=torch.long), cut.long(),
                        torch.full((1,), n, device=deg.device, dtype=torch.long)])
    starts = torch.maximum(starts, torch.cummax(starts, 0).values)
    return starts.cpu()


@dataclass
class SideLayout:
    n: int                 # global dense rows
    starts: torch.Tensor   # [world+1] dense row ranges (cpu int64)
    rows_per_rank: int     # padded rows per rank
    dense_map: torch.Tensor  # id -> dense row (-1 absent), device int32
    uniq: torch.Tensor       # dense row -> id, device int32

    def owner_of(self, dense: torch.Tensor) -> torch.Tensor:
        st = self.starts.to(dense.device)
        return torch.searchsorted(st[1:-1].contiguous(), dense.long(), right=True)

    def padded(self, dense: torch.Tensor) -> torch.Tensor:
        o = self.owner_of(dense)
        st = self.starts.to(dense.device)
        return (o * self.rows_per_rank + (dense.long() - st[o])).to(torch.int32)


class ShardedALS:
    """ALS with users and items sharded over the ranks of `group`."""

    def __init__(self, users, items, ratings, device=None, group=None, kernels=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
            else torch.device("cpu"))
        self.K = kernels if kernels is not None else HipKernels(self.device)
        dev = self.device
        u = torch.as_tensor(users).to(dev, torch.int32)
        i = torch.as_tensor(items).to(dev, torch.int32)
        r = torch.as_tensor(ratings).to(dev, torch.float32)
        self.local_nnz = int(u.numel())
        mx = torch.tensor([int(u.max()) if u.numel() else -1, int(i.max()) if i.numel() else -1],
                          dtype=torch.int64, device=dev)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
        u_space, i_space = int(mx[0]) + 1, int(mx[1]) + 1
        self.users = self._layout(u, u_space)
        self.items = self._layout(i, i_space)
        nz = torch.tensor([self.local_nnz], dtype=torch.int64, device=dev)
        dist.all_reduce(nz, group=group)
        self.nnz = int(nz)
        # dense -> padded global numbering of both sides
        ud = self.users.dense_map[u.long()]
        idn = self.items.dense_map[i.long()]
        u_pad, i_pad = self.users.padded(ud), self.items.padded(idn)
        # route each rating to its user owner and to its item owner (one-time all_to_all)
        ru, rc, rv = self._route(self.users.owner_of(ud), u_pad, i_pad, r)
        self.user_rows = self._local_rows(self.users)
        self.user_block = self.K.build_block(
            ru - self.rank * self.users.rows_per_rank, rc, rv, self.user_rows,
            self.world * self.items.rows_per_rank)
        ri_, rc_, rv_ = self._route(self.items.owner_of(idn), i_pad, u_pad, r)
        self.item_rows = self._local_rows(self.items)
        self.item_block = self.K.build_block(
            ri_ - self.rank * self.items.rows_per_rank, rc_, rv_, self.item_rows,
            self.world * self.users.rows_per_rank)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.rank_k = 0

    # ---- setup helpers ----
    def _layout(self, ids: torch.Tensor, space: int) -> SideLayout:
        dev = self.device
        flag = torch.zeros(space, dtype=torch.int32, device=dev)
        flag[ids.long()] = 1
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        present = torch.nonzero(flag).flatten().to(torch.int32)
        dmap, uniq, n = self.K.index_build(present, space)
        deg = torch.zeros(n, dtype=torch.int64, device=dev)
        deg.index_add_(0, dmap[ids.long()].long(), torch.ones_like(ids, dtype=torch.int64))
        dist.all_reduce(deg, group=self.group)
        starts = _ranges(deg, self.world)
        rpr = max(int((starts[1:] - starts[:-1]).max()), 1)
        return SideLayout(n, starts, rpr, dmap, uniq)

    def _local_rows(self, side: SideLayout) -> int:
        return int(side.starts[self.rank + 1] - side.starts[self.rank])

    def _route(self, dest: torch.Tensor, a: torch.Tensor, b: torch.Tensor, v: torch.Tensor):
        order = torch.argsort(dest, stable=True)
        send_counts = torch.bincount(dest, minlength=self.world).to(torch.int64)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        sc, rc = send_counts.tolist(), recv_counts.tolist()
        out = []
        for t in (a, b, v):
            t = t[order].contiguous()
            o = torch.empty(sum(rc), dtype=t.dtype, device=t.device)
            dist.all_to_all_single(o, t, rc, sc, group=self.group)
            out.append(o)
        return out

    # ---- ALS ----
    def init_factors(self, rank: int, seed: int = 0, U0_global: Optional[torch.Tensor] = None):
        """U in the padded layout.  U0_global: optional [n_users_dense, rank] start."""
        self.rank_k = rank
        ld = self.K.ld(rank)
        dev = self.device
        W = self.world
        self.U_full = torch.zeros((W * self.users.rows_per_rank, ld), dtype=torch.float32,
                                  device=dev)
        self.V_full = torch.zeros((W * self.items.rows_per_rank, ld), dtype=torch.float32,
                                  device=dev)
        self.U_loc = torch.zeros((self.users.rows_per_rank, ld), dtype=torch.float32, device=dev)
        self.V_loc = torch.zeros((self.items.rows_per_rank, ld), dtype=torch.float32, device=dev)
        s0 = int(self.users.starts[self.rank])
        n_loc = self.user_rows
        if U0_global is not None:
            U0 = torch.as_tensor(U0_global).to(dev, torch.float32)
            self.U_loc[:n_loc, :rank] = U0[s0:s0 + n_loc]
        else:
            g = torch.Generator(device=dev)
            g.manual_seed((int(seed) * 1000003 + self.rank) & 0x7FFFFFFFFFFFFFFF)
            x = torch.randn((n_loc, rank), generator=g, device=dev)
            self.U_loc[:n_loc, :rank] = x / torch.linalg.vector_norm(x, dim=1, keepdim=True)
        dist.all_gather_into_tensor(self.U_full, self.U_loc, group=self.group)

    def _yty(self, full: torch.Tensor, loc: torch.Tensor, n_loc: int):
        g = self.K.yty(loc, n_loc, self.rank_k)
        dist.all_reduce(g, group=self.group)
        return g

    def half_sweep_items(self, reg, implicit=False, alpha=1.0):
        yty = self._yty(self.U_full, self.U_loc, self.user_rows) if implicit else None
        self.K.solve_half(self.item_block, self.U_full, self.V_loc, self.rank_k, reg, implicit,
                          alpha, yty, self.status)
        dist.all_gather_into_tensor(self.V_full, self.V_loc, group=self.group)

    def half_sweep_users(self, reg, implicit=False, alpha=1.0):
        yty = self._yty(self.V_full, self.V_loc, self.item_rows) if implicit else None
        self.K.solve_half(self.user_block, self.V_full, self.U_loc, self.rank_k, reg, implicit,
                          alpha, yty, self.status)
        dist.all_gather_into_tensor(self.U_full, self.U_loc, group=self.group)

    def iterate(self, reg, implicit=False, alpha=1.0):
        self.half_sweep_items(reg, implicit, alpha)
        self.half_sweep_users(reg, implicit, alpha)

    def fit(self, rank, max_iter, reg, implicit=False, alpha=1.0, seed=0, U0_global=None):
        self.init_factors(rank, seed, U0_global)
        self.status.zero_()
        for _ in range(max_iter):
            self.iterate(reg, implicit, alpha)
        st = self.status.clone()
        dist.all_reduce(st, op=dist.ReduceOp.MAX, group=self.group)
        if int(st) != 0:
            raise RuntimeError("Cholesky failed (non-positive pivot) on some rank")
        return self

    # ---- factor views in dense order (replicated on every rank) ----
    def _dense_rows(self, side: SideLayout, full: torch.Tensor) -> torch.Tensor:
        dense = torch.arange(side.n, device=full.device)
        return full[side.padded(dense).long(), :self.rank_k]

    def user_factors(self):
        return self.users.uniq, self._dense_rows(self.users, self.U_full)

    def item_factors(self):
        return self.items.uniq, self._dense_rows(self.items, self.V_full)
