"""One-process-per-GPU sharded ALS over torch.distributed (RCCL on ROCm).

Replaces Spark's data movement on the ALS path (SURVEY.md §2 "Spark
data-movement site" table, §8e):
  * partitionRatings / makeBlocks shuffles   -> one-time all_to_all(v) that routes
    every rating to the rank owning its user row and to the rank owning its
    item row;
  * computeFactors' srcOut.groupByKey        -> all_gathers of the updated factor
    half (factors are replicated; each rank solves only its own rows), issued
    per row chunk and overlapped with the solve of the next chunk;
  * computeYtY's treeAggregate (implicit)    -> local YtY of the rank's own rows +
    all_reduce of the k_pad^2 fp64 Gram;
  * computeError's reduce + count (RecommenderSystem.py:123, :126)
                                             -> local fused (sse, n) + all_reduce;
  * predict / recommendForAll                -> local: the factors are replicated
    after every half-sweep, so no collective (each rank scores its own users).

Rows are split into contiguous, nnz-balanced ranges of the global dense index
(no row is split across ranks), and each rank's range into C nnz-balanced
chunks.  Every factor matrix lives in a *padded* global layout
[C, world, rows_per_chunk, ld]: row `d` in chunk `c` of owner `o` sits at
`(c * world + o) * rows_per_chunk + (d - chunk_start[o][c])`, so chunk c of
every rank is one contiguous all_gather_into_tensor target, the gathered
buffer is directly the gather table of the next half-sweep (no unpacking
copy), and CSR column indices are stored in that padded numbering.  A
half-sweep solves chunk c, then starts its all-gather (async, RCCL's stream)
while chunk c+1 is solved; the waits come before the next half-sweep.

The initial factors are drawn from the seed over the GLOBAL dense user rows
(exactly ALSCore.init_factors' draw) and each rank keeps its slice, so a fit is
independent of the world size.

The arithmetic is delegated to a `kernels` object (default: the HIP kernels of
libals_hip.so).  Tests substitute the CPU oracle to check the coordination
logic with the gloo backend on CPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .engine import id_offset


class HipKernels:
    """The product kernels (libals_hip.so) behind the interface ShardedALS uses.

    chunk: ratings per heavy-row task; None = the single-GPU engine's choice per fit
    (engine.chunk_for(rank, implicit): 16384 for explicit fits at rank > 64, else 4096),
    applied by ShardedALS rescheduling its blocks when a fit asks for another length."""

    def __init__(self, device, chunk: Optional[int] = None):
        from . import engine as E
        self.E = E
        self.device = torch.device(device)
        self.ws = E.Workspace(self.device)
        self.auto_chunk = chunk is None
        self.chunk = chunk or E.DEFAULT_CHUNK
        self.max_chunks = 0  # heavy-row chunks of the largest block: one workspace layout
        self.max_rows = 0    # rows of the largest block (rescue list)
        # the pipelined (two-segment) item side: one workspace for every item chunk, the
        # chunks' slots in disjoint ranges, one Y prep per part (engine.solve_half_split)
        self.split_ws = E.Workspace(self.device)
        self.split_slots = 0
        self.split_rows = 0

    def chunk_for(self, rank: int, implicit: bool) -> int:
        return self.E.chunk_for(rank, implicit) if self.auto_chunk else self.chunk

    def reschedule(self, block, chunk: int):
        """The same CSR block with `chunk`-rating heavy-row tasks."""
        blk = self.E.schedule_block(block.n_rows, block.nnz, block.row_ptr, block.col, block.val,
                                    self.ws, chunk)
        self.max_chunks = max(self.max_chunks, blk.n_chunks)
        self.max_rows = max(self.max_rows, blk.n_light + blk.n_heavy)
        return blk

    def block_chunk(self, block) -> int:
        return block.chunk

    def index_build(self, ids: torch.Tensor, id_space: int):
        idx = self.E.build_index(ids.to(self.device, torch.int32).contiguous(), id_space, self.ws)
        return idx.map, idx.uniq, idx.n

    def build_block(self, rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor,
                    n_rows: int, n_cols: int, chunk: Optional[int] = None):
        ident_r = torch.arange(max(n_rows, 1), dtype=torch.int32, device=self.device)
        ident_c = torch.arange(max(n_cols, 1), dtype=torch.int32, device=self.device)
        ri = self.E.IdIndex(ident_r, ident_r, n_rows)
        ci = self.E.IdIndex(ident_c, ident_c, n_cols)
        blk = self.E.build_block(rows.contiguous(), ri, cols.contiguous(), ci,
                                 vals.contiguous(), self.ws, chunk or self.chunk)
        self.max_chunks = max(self.max_chunks, blk.n_chunks)
        self.max_rows = max(self.max_rows, blk.n_light + blk.n_heavy)
        return blk

    def yty(self, Y: torch.Tensor, n: int, rank: int) -> torch.Tensor:
        return self.E.compute_yty(Y, n, rank, self.ws)

    def solve_half(self, block, Y, X, rank, reg, implicit, alpha, yty, status, first=True):
        """first=False: Y was prepared (scale, split table) by the previous call of this
        half-sweep; only this block's rating scale and launches run."""
        E = self.E
        E.solve_half(block, Y, X, rank, reg, implicit, alpha, yty, status, self.ws,
                     phases=E.PHASE_ALL if first else E.PHASE_ALL & ~E.PHASE_PREP,
                     ws_chunks=self.max_chunks, ws_rows=self.max_rows)

    def split_schedule(self, block, seg, n_src_early: int, slot_base: int = 0):
        """Two-segment schedule of an item block (pipelined item half-sweep), its slots
        numbered from slot_base (the item chunks share one workspace)."""
        sched = self.E.split_schedule(block, seg, n_src_early, block.chunk, slot_base)
        self.split_slots = max(self.split_slots, sched.n_slots)
        self.split_rows = max(self.split_rows, block.n_rows)
        return sched

    def split_slot_end(self, sched) -> int:
        return sched.n_slots

    def solve_split(self, block, sched, part, Y, X, rank, reg, implicit, alpha, yty, status,
                    first: bool):
        """One part ("early" / "late") of a two-segment half-sweep on the shared item
        workspace; first: the first item chunk of this part (it preps Y for them all)."""
        self.E.solve_half_split(block, sched, part, Y, X, rank, reg, implicit, alpha, yty,
                                status, self.split_ws, prep=first, ws_slots=self.split_slots,
                                ws_rows=self.split_rows)

    def predict(self, u_keys, i_keys, umap, imap, U, V, rank) -> torch.Tensor:
        E = self.E
        return E.predict_pairs(u_keys, i_keys, E.IdIndex(umap, umap, 0), E.IdIndex(imap, imap, 0),
                               U, V, rank)

    def rmse_partial(self, u_keys, i_keys, r, umap, imap, U, V, rank) -> torch.Tensor:
        E = self.E
        return E.rmse_pairs(u_keys, i_keys, r, E.IdIndex(umap, umap, 0),
                            E.IdIndex(imap, imap, 0), U, V, rank, self.ws)

    def topk(self, Q, n_q, V, n_v, rank, top):
        return self.E.topk_rows(Q, n_q, V, n_v, rank, top)

    def ld(self, rank: int) -> int:
        return self.E.ld_for(rank)

    def block_values(self, block) -> torch.Tensor:
        return block.val


# Largest message of one collective call.  The factor all-gathers and the one-time
# rating routing at configs[3] scale move several GB per call; every call is kept
# at or below this, and _guard() refuses a call above it before it is issued.
# (The round-2 fault: at 1e9 ratings on one rank the uncapped routing all_to_all
# moved 1e9 int32 = 4.0e9 bytes per call — 1e9 elements is below 2^31, the byte
# count 4.0e9 is above 2^31 - 1 — and faulted inside RCCL; capped at 1 GiB the same
# routing runs.  DESIGN.md §6.)
MAX_COLLECTIVE_BYTES = 1 << 30
# Row weight in ratings-equivalents for the range balance: a row's solve costs as
# much as the Gram of a few hundred ratings, so ranges balance deg + ROW_WEIGHT.
ROW_WEIGHT = 256
# No range holds more than PAD_CAP x the mean rows per range: the replicated factor
# tables and the all-gathers are padded to the largest range.
PAD_CAP = 1.25


def _guard(nbytes: int, what: str) -> None:
    """Refuse a collective above MAX_COLLECTIVE_BYTES (every rank computes the same
    sizes, so every rank raises before any of them issues the call)."""
    if nbytes > MAX_COLLECTIVE_BYTES:
        raise RuntimeError(f"{what}: {nbytes} bytes in one collective call exceeds "
                           f"MAX_COLLECTIVE_BYTES = {MAX_COLLECTIVE_BYTES} (use more chunks)")


def _capped_pieces(t: torch.Tensor, what: str):
    """1-D views of the contiguous tensor t of at most MAX_COLLECTIVE_BYTES each (every
    rank holds the same shape, so every rank issues the same calls)."""
    if not t.is_contiguous():
        raise ValueError(f"{what}: collective on a non-contiguous tensor")
    flat = t.view(-1)
    per = max(1, MAX_COLLECTIVE_BYTES // t.element_size())
    for s in range(0, flat.numel(), per):
        piece = flat[s:s + per]
        _guard(piece.numel() * piece.element_size(), what)
        yield piece


def all_reduce_capped(t: torch.Tensor, what: str, op=None, group=None) -> torch.Tensor:
    """dist.all_reduce of t in place, split into calls of <= MAX_COLLECTIVE_BYTES (the
    id-space flag and degree arrays of the setup grow with the id range: 2^31 ids would
    be an 8 GiB int32 all_reduce in one call)."""
    op = dist.ReduceOp.SUM if op is None else op
    for piece in _capped_pieces(t, what):
        dist.all_reduce(piece, op=op, group=group)
    return t


def broadcast_capped(t: torch.Tensor, src: int, what: str, group=None) -> torch.Tensor:
    """dist.broadcast of t in place in calls of <= MAX_COLLECTIVE_BYTES (checkpointed
    factor tables: 10M x 128 fp32 = 5.1 GB)."""
    for piece in _capped_pieces(t, what):
        dist.broadcast(piece, src=src, group=group)
    return t


def _ranges(deg: torch.Tensor, parts: int, cap_rows: Optional[int] = None):
    """Contiguous row ranges start[w] .. start[w+1], w < parts, balancing deg + ROW_WEIGHT
    (no row is split), with at most cap_rows rows per range (default ceil(PAD_CAP x
    n / parts)) — when row ids correlate with popularity, pure nnz balance would give
    the tail range most of the rows and every replicated table that padding."""
    n = deg.numel()
    if cap_rows is None:
        cap_rows = math.ceil(PAD_CAP * n / parts) if n else 1
    cap_rows = max(int(cap_rows), 1)
    w8 = deg.to(torch.float64) + float(ROW_WEIGHT)
    cum = torch.cumsum(w8, 0)
    total = float(cum[-1]) if n else 0.0
    targets = torch.tensor([total * w / parts for w in range(1, parts)], dtype=torch.float64,
                           device=deg.device)
    cut = (torch.searchsorted(cum, targets, right=True) if n else
           torch.zeros(parts - 1, dtype=torch.long)).cpu().tolist()
    starts = [0]
    for w in range(1, parts):
        lo = max(starts[-1], n - (parts - w) * cap_rows)  # the rest must fit the rest
        hi = min(starts[-1] + cap_rows, n)
        starts.append(min(max(int(cut[w - 1]), lo), hi))
    starts.append(n)
    return torch.tensor(starts, dtype=torch.long)


@dataclass
class SideLayout:
    n: int                 # global dense rows
    starts: torch.Tensor   # [world+1] dense row ranges of the ranks (cpu int64)
    cstarts: torch.Tensor  # [world, C+1] dense row ranges of each rank's chunks (cpu int64)
    rows_per_chunk: int    # padded rows per (chunk, rank)
    dense_map: torch.Tensor  # (id - offset) -> dense row (-1 absent), device int32
    uniq: torch.Tensor       # dense row -> id - offset, device int32
    offset: int = 0          # ids are keyed as id - offset (engine.id_offset)
    _pmap: Optional[torch.Tensor] = None

    @property
    def chunks(self) -> int:
        return self.cstarts.shape[1] - 1

    @property
    def rows_per_rank(self) -> int:
        return self.chunks * self.rows_per_chunk

    def ids(self) -> torch.Tensor:
        return self.uniq if self.offset == 0 else (self.uniq.long() + self.offset).to(torch.int32)

    def keys(self, ids: torch.Tensor) -> torch.Tensor:
        """ids -> map keys (-1 outside the mapped range)."""
        s = ids.long() - self.offset
        return torch.where((s >= 0) & (s < self.dense_map.numel()), s, -1).to(torch.int32)

    def owner_of(self, dense: torch.Tensor) -> torch.Tensor:
        st = self.starts.to(dense.device)
        return torch.searchsorted(st[1:-1].contiguous(), dense.long(), right=True)

    def padded(self, dense: torch.Tensor) -> torch.Tensor:
        """Position of dense rows in the [C, world, rows_per_chunk] layout."""
        W, C = self.cstarts.shape[0], self.chunks
        b = self.cstarts[:, :C].reshape(-1).to(dense.device)  # chunk starts, rank-major
        g = torch.searchsorted(b, dense.long(), right=True) - 1  # last chunk starting <= d
        o, c = g // C, g % C
        return ((c * W + o) * self.rows_per_chunk + (dense.long() - b[g])).to(torch.int32)

    def padded_map(self) -> torch.Tensor:
        """(id - offset) -> padded row (-1 absent): the id map of the replicated tables."""
        if self._pmap is None:
            d = self.dense_map
            pm = torch.full_like(d, -1)
            ok = d >= 0
            pm[ok] = self.padded(d[ok])
            self._pmap = pm
        return self._pmap

    def chunk_rows(self, rank: int, c: int) -> int:
        return int(self.cstarts[rank, c + 1] - self.cstarts[rank, c])

    @property
    def padding(self) -> float:
        """Rows of the replicated (padded) table / real rows (<= PAD_CAP by _ranges)."""
        world = self.cstarts.shape[0]
        return world * self.rows_per_rank / max(self.n, 1)


class ShardedALS:
    """ALS with users and items sharded over the ranks of `group`."""

    def __init__(self, users, items, ratings, device=None, group=None, kernels=None,
                 chunks: Optional[int] = None, pipeline=None, exchange: str = "ring"):
        """pipeline: the pipelined item half-sweep (below).  None / False: off (the
        default until an A/B on a multi-GPU node shows it pays: no such node has been
        available to this build); True: on; "auto": on when the exchange model
        (pipeline_pays) says so at the fit's rank.
        exchange: how a solved factor chunk reaches every rank — "ring": RCCL's
        all_gather_into_tensor; "peers": one batched isend / irecv per peer (every rank
        sends its chunk to all W - 1 peers at once, so all xGMI links carry traffic
        instead of the ring's one in / one out link per step; unmeasured on a
        multi-GPU node)."""
        if exchange not in ("ring", "peers"):
            raise ValueError(f"exchange must be 'ring' or 'peers', got {exchange!r}")
        if pipeline not in (None, False, True, "auto"):
            raise ValueError(f"pipeline must be None, False, True or 'auto', got {pipeline!r}")
        self.exchange = exchange
        self.group = group
        self.proc = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        # row chunks per rank: the all-gather of chunk c overlaps the solve of c+1.
        # Each chunk is its own launch (its own tail): measured +0.15 ms per
        # iteration per extra chunk at the ML-25M shape on one GPU, so chunking
        # pays only when the exchanged factor half is large (_auto_chunks).
        self._chunks_arg = int(chunks) if chunks else None
        self.chunks = 1
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
            else torch.device("cpu"))
        self.K = kernels if kernels is not None else HipKernels(self.device)
        dev = self.device
        u = torch.as_tensor(users).to(dev, torch.int32)
        i = torch.as_tensor(items).to(dev, torch.int32)
        r = torch.as_tensor(ratings).to(dev, torch.float32)
        self.local_nnz = int(u.numel())
        big = 1 << 40
        mm = torch.tensor([int(u.max()) if u.numel() else -big, int(i.max()) if i.numel() else -big,
                           -int(u.min()) if u.numel() else -big,
                           -int(i.min()) if i.numel() else -big], dtype=torch.int64, device=dev)
        all_reduce_capped(mm, "id range", dist.ReduceOp.MAX, group)
        (umax, imax), (umin, imin) = mm[:2].tolist(), (-mm[2:]).tolist()
        if umax < umin:
            raise ValueError("ALS needs at least one rating")
        uoff, ioff = id_offset(umin, umax), id_offset(imin, imax)
        u_space, i_space = umax - uoff + 1, imax - ioff + 1
        if uoff:
            u = (u.long() - uoff).to(torch.int32)
        if ioff:
            i = (i.long() - ioff).to(torch.int32)
        self.chunks = self._chunks_arg or self._auto_chunks(u_space, i_space)
        self.users = self._layout(u, u_space, uoff)
        self.items = self._layout(i, i_space, ioff)
        nz = torch.tensor([self.local_nnz], dtype=torch.int64, device=dev)
        all_reduce_capped(nz, "rating count", group=group)
        self.nnz = int(nz)
        # dense -> padded global numbering of both sides
        ud = self.users.dense_map[u.long()]
        idn = self.items.dense_map[i.long()]
        u_pad, i_pad = self.users.padded(ud), self.items.padded(idn)
        # route each rating to its user owner and to its item owner (one-time all_to_all)
        ru, rc, rv = self._route(self.users.owner_of(ud), u_pad, i_pad, r)
        self.user_rows = self._local_rows(self.users)
        self.user_blocks = self._blocks(self.users, ru, rc, rv, self.items)
        ri_, rc_, rv_ = self._route(self.items.owner_of(idn), i_pad, u_pad, r)
        self.item_rows = self._local_rows(self.items)
        self.item_nnz = int(ri_.numel())
        # pipelined item half-sweep: each item row's ratings are split into the users of
        # chunks 0..C-2 (early) and of chunk C-1 (late), so the early partial normal
        # equations are formed while the last user chunk's all-gather is still in
        # flight (_pipelined_items).  The item blocks are built early-first whenever it
        # may run; whether it does is settled per fit (init_factors: "auto" asks the
        # exchange model at the fit's rank).
        self._pipeline_arg = pipeline
        # (True also at one rank, where it only exercises the two-segment kernels)
        can_split = bool(pipeline) and self.users.chunks >= 2
        self.pipeline = False
        self.item_split = None
        self._item_segs = None
        self.item_blocks = self._blocks(self.items, ri_, rc_, rv_, self.users, split=can_split)
        self._pending_u = []  # async all-gathers of U chunks not yet waited for
        self._yty_u = None    # YtY of the final U (implicit, pipelined): formed early
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.rank = 0  # factor rank (k); the process rank is self.proc
        self._dense_cache = {}

    # ---- setup helpers ----
    # exchange model of the pipelining choice (unmeasured on a multi-GPU
    # node): a ring all-gather over xGMI at RING_GBS per rank, partial slots at HBM_GBS
    RING_GBS = 150.0
    HBM_GBS = 5000.0

    @classmethod
    def pipeline_cost(cls, world: int, chunks: int, user_rows_per_chunk: int, item_rows: int,
                      item_nnz: int, rank: int, item_chunks: int = 1,
                      chunk: Optional[int] = None) -> dict:
        """The exchange model of the pipelining choice, per item half-sweep (seconds):
        hidden = U chunk C-1's all-gather, (W - 1) x a chunk's rows per rank, which the
        early item partials hide; added = the partial-slot traffic (every item row
        through the slot path: about three passes over one slot per <= chunk-rating
        segment, two segments per row) plus the extra Y prep (one over the arrived prefix
        of U for the early part, beside the one every half-sweep does: read U, write
        its split table)."""
        from . import engine as E
        chunk = chunk or E.DEFAULT_CHUNK
        ld = (rank + 3) // 4 * 4
        kp = 16 * (1 if rank <= 16 else (2 if rank <= 32 else (4 if rank <= 64 else 8)))
        cn = kp // 16
        recv = (world - 1) * user_rows_per_chunk * ld * 4
        segs = 2 * max(item_rows, 1) + item_nnz // chunk
        slot = (cn * (cn + 1) // 2 * 4 + cn + 1) * 64 * 4
        n_u = world * chunks * user_rows_per_chunk
        prep = n_u * (ld + kp) * 4 * (chunks - 1) / max(chunks, 1)
        return {"hidden_s": recv / (cls.RING_GBS * 1e9),
                "added_s": (3 * segs * slot + prep) / (cls.HBM_GBS * 1e9)}

    @classmethod
    def pipeline_pays(cls, world: int, chunks: int, user_rows_per_chunk: int,
                      item_rows: int, item_nnz: int, rank: int = 128, item_chunks: int = 1,
                      chunk: Optional[int] = None) -> bool:
        """Pipeline the item half-sweep when the exchange it hides costs more than twice
        what it adds (pipeline_cost)."""
        if world < 2 or chunks < 2:
            return False
        c = cls.pipeline_cost(world, chunks, user_rows_per_chunk, item_rows, item_nnz, rank,
                              item_chunks, chunk)
        return c["added_s"] < 0.5 * c["hidden_s"]

    def _pipeline_pays(self, rank: int, implicit: bool = False) -> bool:
        """pipeline_pays for this rank's item rows at the fit's rank and task length,
        agreed by every rank (MIN)."""
        chunk = self.K.chunk_for(rank, implicit) if hasattr(self.K, "chunk_for") else None
        ok = self.pipeline_pays(self.world, self.users.chunks, self.users.rows_per_chunk,
                                self.item_rows, self.item_nnz, rank, self.items.chunks, chunk)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=self.device)
        all_reduce_capped(flag, "pipeline choice", dist.ReduceOp.MIN, self.group)
        return bool(int(flag))

    def _settle_pipeline(self, rank: int, implicit: bool = False) -> None:
        """Whether this fit pipelines the item half-sweep (the item blocks were built
        early-first at setup when it may)."""
        arg = self._pipeline_arg
        if self._item_segs is None or not arg:
            self.pipeline = False
        elif arg == "auto":
            self.pipeline = self._pipeline_pays(rank, implicit)
        else:
            self.pipeline = True

    def _schedule_for(self, implicit: bool) -> None:
        """The heavy-row task length of this fit (HipKernels.chunk_for: the single-GPU
        engine's choice) for every block; the pipelined item side's two-segment
        schedules are rebuilt with it."""
        if not hasattr(self.K, "reschedule") or self.rank == 0:
            return
        chunk = self.K.chunk_for(self.rank, implicit)
        blocks = [b for b in self.user_blocks + self.item_blocks if b is not None]
        if all(self.K.block_chunk(b) == chunk for b in blocks):
            return
        self.user_blocks = [None if b is None else self.K.reschedule(b, chunk)
                            for b in self.user_blocks]
        self.item_blocks = [None if b is None else self.K.reschedule(b, chunk)
                            for b in self.item_blocks]
        if self._item_segs is not None:
            self._split_schedules()

    def _split_schedules(self) -> None:
        """Two-segment schedules of the item blocks, slot ranges disjoint (one shared
        workspace, one Y prep per part)."""
        n_src_early = (self.users.chunks - 1) * self.world * self.users.rows_per_chunk
        self.item_split = []
        base = 0
        for blk, seg in zip(self.item_blocks, self._item_segs):
            sched = None
            if blk is not None:
                sched = self.K.split_schedule(blk, seg, n_src_early, base)
                base = self.K.split_slot_end(sched) if hasattr(self.K, "split_slot_end") else 0
            self.item_split.append(sched)
    def _auto_chunks(self, u_space: int, i_space: int) -> int:
        """4 row chunks when a rank's share of the larger id space reaches 1M rows
        (the all-gather then moves >= 256 MB per rank at rank 64); 2 from 4 ranks on
        when the share reaches 64k rows (the weak-scaled configs[1] shape: at 8 ranks
        each receives ~290 MB of U per iteration, about the half-sweep's own time on a
        ring over xGMI, so chunk 0's gather hides behind chunk 1's solve — a model
        choice, the 1-rank cost of the second chunk is +0.15 ms); else 1; and at
        least enough chunks that one chunk's all-gather stays within
        MAX_COLLECTIVE_BYTES: a chunk holds at most ceil(PAD_CAP n / (W C)) rows of each
        rank (the cap _layout applies), so the all-gather of one chunk moves at most
        W x that x 512 B (rank <= 128 factors) — counted exactly, so the guard in
        _solve_and_gather never stops a configuration more chunks would handle."""
        big = max(u_space, i_space)
        W = self.world
        c = 4 if (W > 1 and big // W >= (1 << 20)) else (2 if (W >= 4 and big // W >= (1 << 16)) else 1)
        # (a chunk of one row per rank is the floor: below it the guard decides, with
        # the real row size)
        while (math.ceil(PAD_CAP * big / (W * c)) > 1 and
               W * math.ceil(PAD_CAP * big / (W * c)) * 512 > MAX_COLLECTIVE_BYTES):
            c += 1
        return c

    def _layout(self, ids: torch.Tensor, space: int, offset: int) -> SideLayout:
        dev = self.device
        flag = torch.zeros(space, dtype=torch.int32, device=dev)
        flag[ids.long()] = 1
        all_reduce_capped(flag, "id flags", dist.ReduceOp.MAX, self.group)
        present = torch.nonzero(flag).flatten().to(torch.int32)
        del flag
        dmap, uniq, n = self.K.index_build(present, space)
        deg = torch.zeros(n, dtype=torch.int64, device=dev)
        deg.index_add_(0, dmap[ids.long()].long(), torch.ones_like(ids, dtype=torch.int64))
        all_reduce_capped(deg, "row degrees", group=self.group)
        starts = _ranges(deg, self.world)
        degc = deg.cpu()
        # chunk ranges capped against the GLOBAL mean rows per (rank, chunk), so the
        # padded chunk stays within PAD_CAP of it too
        cap_c = max(1, math.ceil(PAD_CAP * n / (self.world * self.chunks)))
        cst = torch.stack([_ranges(degc[int(starts[w]):int(starts[w + 1])], self.chunks, cap_c)
                           + starts[w] for w in range(self.world)])
        rpc = max(int((cst[:, 1:] - cst[:, :-1]).max()), 1)
        return SideLayout(n, starts, cst, rpc, dmap, uniq, offset)

    def _local_rows(self, side: SideLayout) -> int:
        return int(side.starts[self.proc + 1] - side.starts[self.proc])

    def _blocks(self, side: SideLayout, rows_pad, cols_pad, vals, other: SideLayout,
                split: bool = False):
        """Per-chunk rating blocks of this rank's rows (rows_pad: padded positions).
        split: order every row's ratings early-first — columns (padded rows of `other`)
        in its chunks 0..C-2, then those in its last chunk (the CSR build is stable) —
        and keep each block's two-segment schedule in self.item_split."""
        W, rpc = self.world, side.rows_per_chunk
        late = None
        if split:
            late = (cols_pad.long() // (W * other.rows_per_chunk)) == other.chunks - 1
            order = torch.argsort(late.to(torch.int8), stable=True)
            rows_pad, cols_pad, vals, late = rows_pad[order], cols_pad[order], vals[order], \
                late[order]
            self._item_segs = []
        p = rows_pad.long()
        c = p // (W * rpc)
        j = (p % rpc).to(torch.int32)
        out = []
        for cc in range(side.chunks):
            n_c = side.chunk_rows(self.proc, cc)
            sel = c == cc
            blk = self.K.build_block(j[sel], cols_pad[sel], vals[sel], n_c,
                                     W * other.rows_per_rank) if n_c > 0 else None
            out.append(blk)
            if split:
                seg = None
                if blk is not None:
                    ne = torch.bincount(j[sel & ~late].long(), minlength=n_c)
                    seg = self._row_starts(blk, n_c) + ne.to(torch.int64)
                self._item_segs.append(seg)
        if split:
            self.item_blocks = out
            self._split_schedules()
        return out

    def _row_starts(self, blk, n_rows: int) -> torch.Tensor:
        rp = blk.row_ptr if hasattr(blk, "row_ptr") else torch.as_tensor(blk[0])
        return rp[:n_rows].to(self.device, torch.int64)

    def _route(self, dest: torch.Tensor, a: torch.Tensor, b: torch.Tensor, v: torch.Tensor):
        order = torch.argsort(dest, stable=True)
        send_counts = torch.bincount(dest, minlength=self.world).to(torch.int64)
        recv_counts = torch.empty_like(send_counts)
        _guard(send_counts.numel() * send_counts.element_size(), "routing counts")
        dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        sc, rc = send_counts.tolist(), recv_counts.tolist()
        out = []
        for t in (a, b, v):
            t = t[order].contiguous()
            out.append(self._all_to_all_v(t, sc, rc, send_counts.device))
        return out

    def _all_to_all_v(self, t: torch.Tensor, sc, rc, dev) -> torch.Tensor:
        """all_to_all_single in rounds: round j moves elements [j*C, (j+1)*C) of every
        peer segment, with C chosen so one call stays within MAX_COLLECTIVE_BYTES.
        The round count is the max over ranks (every rank issues the same calls)."""
        W = self.world
        o = torch.empty(sum(rc), dtype=t.dtype, device=t.device)
        # per-peer elements per round: one round moves at most W x per elements, so every
        # call is within MAX_COLLECTIVE_BYTES by construction (tested with gloo)
        per = max(1, MAX_COLLECTIVE_BYTES // (t.element_size() * W))
        rounds_t = torch.tensor([-(-max(max(sc), max(rc), 1) // per)], dtype=torch.int64,
                                device=dev)
        all_reduce_capped(rounds_t, "routing rounds", dist.ReduceOp.MAX, self.group)
        rounds = max(1, int(rounds_t.item()))
        if rounds == 1:
            dist.all_to_all_single(o, t, rc, sc, group=self.group)
            return o
        soff = [sum(sc[:w]) for w in range(W)]
        roff = [sum(rc[:w]) for w in range(W)]
        for j in range(rounds):
            s_ = [max(0, min(per, sc[w] - j * per)) for w in range(W)]
            r_ = [max(0, min(per, rc[w] - j * per)) for w in range(W)]
            send = torch.cat([t[soff[w] + j * per: soff[w] + j * per + s_[w]] for w in range(W)])
            recv = torch.empty(sum(r_), dtype=t.dtype, device=t.device)
            dist.all_to_all_single(recv, send, r_, s_, group=self.group)
            pos = 0
            for w in range(W):
                o[roff[w] + j * per: roff[w] + j * per + r_[w]] = recv[pos: pos + r_[w]]
                pos += r_[w]
        return o

    @property
    def n_users(self) -> int:
        return self.users.n

    @property
    def n_items(self) -> int:
        return self.items.n

    # ---- ALS ----
    def init_factors(self, rank: int, seed: int = 0, U0=None, U0_global=None):
        """U in the padded layout.  The default draw is ALSCore.init_factors' one over
        all global dense user rows (unit-norm Gaussian rows from `seed`), sliced to
        this rank's rows; U0 / U0_global: an explicit [n_users_dense, rank] start."""
        U0 = U0 if U0 is not None else U0_global
        self._drain()
        self._yty_u = None
        self.rank = rank
        self._settle_pipeline(rank)
        self._dense_cache = {}
        ld = self.K.ld(rank)
        dev = self.device
        W = self.world
        us, its = self.users, self.items
        self.U_full = torch.zeros((W * us.rows_per_rank, ld), dtype=torch.float32, device=dev)
        self.V_full = torch.zeros((W * its.rows_per_rank, ld), dtype=torch.float32, device=dev)
        self.U_loc = torch.zeros((us.chunks, us.rows_per_chunk, ld), dtype=torch.float32,
                                 device=dev)
        self.V_loc = torch.zeros((its.chunks, its.rows_per_chunk, ld), dtype=torch.float32,
                                 device=dev)
        cs = us.cstarts[self.proc]
        s0 = int(cs[0])
        n_loc = self.user_rows
        if U0 is not None:
            x = torch.as_tensor(U0).to(dev, torch.float32)[s0:s0 + n_loc, :rank]
        else:
            g = torch.Generator(device=dev)
            g.manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
            x = torch.randn((us.n, rank), generator=g, device=dev, dtype=torch.float32)
            x = (x / torch.linalg.vector_norm(x, dim=1, keepdim=True))[s0:s0 + n_loc]
        for c in range(us.chunks):
            a, b = int(cs[c]) - s0, int(cs[c + 1]) - s0
            self.U_loc[c, :b - a, :rank] = x[a:b]
        del x
        full = self.U_full.view(us.chunks, -1, ld)
        _guard(full[0].numel() * full.element_size(), "factor all_gather")
        works = []
        for c in range(us.chunks):
            works.extend(self._exchange(full[c], self.U_loc[c]))
        for w in works:
            w.wait()

    def _yty(self, loc: torch.Tensor):
        # local rows of every chunk (padding rows are zero and add nothing), then all_reduce
        g = self.K.yty(loc.view(-1, loc.shape[-1]), loc.shape[0] * loc.shape[1], self.rank)
        g = g.contiguous()
        all_reduce_capped(g, "YtY", group=self.group)
        return g

    def _solve_and_gather(self, blocks, Y_full, X_loc, X_full, reg, implicit, alpha, yty,
                          before_last=None, wait=True):
        """Solve chunk c, start its all-gather, go on with chunk c+1; wait at the end
        (wait=False: return the pending all-gathers).  before_last runs after the last
        chunk's solve, before its all-gather is issued."""
        Xf = X_full.view(X_loc.shape[0], -1, X_full.shape[1])
        _guard(Xf[0].numel() * Xf.element_size(), "factor all_gather")
        works = []
        first = True
        for c, blk in enumerate(blocks):
            if blk is not None:
                self.K.solve_half(blk, Y_full, X_loc[c], self.rank, reg, implicit, alpha, yty,
                                  self.status, first=first)
                first = False
            if before_last is not None and c == len(blocks) - 1:
                before_last()
            works.extend(self._exchange(Xf[c], X_loc[c]))
        self._dense_cache = {}
        if not wait:
            return works
        for w in works:
            w.wait()
        return []

    def _exchange(self, full_c: torch.Tensor, loc_c: torch.Tensor) -> list:
        """Start the exchange of this rank's solved chunk loc_c into full_c ([world, rows,
        ld]: every rank's chunk c) on every rank; returns the pending works.
        "ring": one all_gather_into_tensor (RCCL's ring over xGMI: W - 1 steps, each
        rank's one in / one out link busy per step).  "peers": one batched group of
        isend / irecv, this rank's chunk to each of the W - 1 peers and theirs into
        full_c[peer] (every link at once), the own chunk copied locally."""
        _guard(loc_c.numel() * loc_c.element_size() * self.world, "factor exchange")
        if self.exchange == "ring" or self.world == 1:
            return [dist.all_gather_into_tensor(full_c, loc_c, group=self.group, async_op=True)]
        fv = full_c.view(self.world, *loc_c.shape)
        fv[self.proc].copy_(loc_c)
        ops = []
        for step in range(1, self.world):  # peers in a rotated order: no hot spot at rank 0
            to, frm = (self.proc + step) % self.world, (self.proc - step) % self.world
            ops.append(dist.P2POp(dist.isend, loc_c, self._peer(to), group=self.group))
            ops.append(dist.P2POp(dist.irecv, fv[frm], self._peer(frm), group=self.group))
        return dist.batch_isend_irecv(ops)

    def _peer(self, r: int) -> int:
        """Global rank of process r of self.group."""
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def _drain(self) -> None:
        """Wait for the U all-gathers a pipelined user half-sweep left in flight."""
        for w in self._pending_u:
            w.wait()
        self._pending_u = []

    def _pipelined_items(self, reg, implicit, alpha, yty):
        """Item half-sweep over the two-segment schedules: the early partials of every
        item chunk (ratings of users in U chunks 0..C-2) are formed while U chunk C-1's
        all-gather is still in flight; then, once it has arrived, the late partials, the
        per-row fp64 sums and the solves, each chunk's V all-gather issued behind it."""
        pend = self._pending_u
        for w in pend[:-1]:
            w.wait()
        first = True
        for c, blk in enumerate(self.item_blocks):
            if blk is not None:
                self.K.solve_split(blk, self.item_split[c], "early", self.U_full, self.V_loc[c],
                                   self.rank, reg, implicit, alpha, yty, self.status, first)
                first = False
        for w in pend[-1:]:
            w.wait()
        self._pending_u = []
        Vf = self.V_full.view(self.V_loc.shape[0], -1, self.V_full.shape[1])
        _guard(Vf[0].numel() * Vf.element_size(), "factor all_gather")
        works = []
        first = True
        for c, blk in enumerate(self.item_blocks):
            if blk is not None:
                self.K.solve_split(blk, self.item_split[c], "late", self.U_full, self.V_loc[c],
                                   self.rank, reg, implicit, alpha, yty, self.status, first)
                first = False
            works.extend(self._exchange(Vf[c], self.V_loc[c]))
        for w in works:
            w.wait()
        self._dense_cache = {}

    def half_sweep_items(self, reg, implicit=False, alpha=1.0):
        if implicit:
            yty = self._yty_u if self._yty_u is not None else self._yty(self.U_loc)
        else:
            yty = None
        self._yty_u = None
        if self.pipeline:
            self._pipelined_items(reg, implicit, alpha, yty)
            return
        self._drain()
        self._solve_and_gather(self.item_blocks, self.U_full, self.V_loc, self.V_full, reg,
                               implicit, alpha, yty)

    def half_sweep_users(self, reg, implicit=False, alpha=1.0):
        self._drain()
        yty = self._yty(self.V_loc) if implicit else None
        before_last = None
        if self.pipeline and implicit:
            # the next item half-sweep's YtY of the final U: its all_reduce is issued
            # before U chunk C-1's all-gather, so the early item partials need not wait
            # for that gather
            def before_last():
                self._yty_u = self._yty(self.U_loc)
        self._pending_u = self._solve_and_gather(
            self.user_blocks, self.V_full, self.U_loc, self.U_full, reg, implicit, alpha, yty,
            before_last=before_last, wait=not self.pipeline)

    def iterate(self, reg, implicit=False, alpha=1.0):
        self._schedule_for(implicit)
        self.half_sweep_items(reg, implicit, alpha)
        self.half_sweep_users(reg, implicit, alpha)

    def check_status(self) -> None:
        self._drain()
        # (max, -min) over ranks: a failed row (> 0) and a rescue-list overflow (-1)
        # both reach every rank
        st = torch.cat([self.status, -self.status]).to(torch.int64)
        all_reduce_capped(st, "status", dist.ReduceOp.MAX, self.group)
        hi, neg = int(st[0]), int(st[1])
        if neg > 0:
            raise RuntimeError("als_solve_half rescue list overflow on some rank: the LAUNCH "
                               "phases ran again before the RESCUE phase consumed the list")
        if hi != 0:
            raise RuntimeError("Cholesky failed (non-positive pivot) on some rank: the normal "
                               "equations are not positive definite (Spark raises from dppsv)")

    def fit(self, rank, max_iter, reg, implicit=False, alpha=1.0, seed=0, U0=None,
            U0_global=None, checkpoint_dir=None, checkpoint_interval=10, resume=False):
        """ALSCore.fit's contract.  Checkpoints hold the dense global factors (written
        by process 0, read by every rank), so a job may resume on another world size."""
        from . import checkpoint as C
        init = C.init_key(seed, U0 if U0 is not None else U0_global) if checkpoint_dir else None
        # process 0 decides and broadcasts (start, factors): every rank resumes alike
        start, Uc, Vc = C.resume_point_agreed(checkpoint_dir, resume, self, rank, reg, implicit,
                                              alpha, max_iter, init, self.group, self.device)
        if Uc is not None:
            U0, U0_global = None, Uc
        self.init_factors(rank, seed, U0, U0_global)
        self._settle_pipeline(rank, implicit)
        if Vc is not None:
            self._set_dense(False, Vc)
        self.status.zero_()
        for it in range(start, max_iter):
            self.iterate(reg, implicit, alpha)
            C.maybe_save(checkpoint_dir, checkpoint_interval, it + 1, self, rank, reg, implicit,
                         alpha, writer=self.proc == 0, init=init)
        if checkpoint_dir:
            dist.barrier(group=self.group)
        self.check_status()
        return self

    def _set_dense(self, user_side: bool, F) -> None:
        """Overwrite one replicated factor table (and this rank's rows) from a dense
        [n, rank] host/device array (every rank passes the same array)."""
        self._drain()
        side, full, loc = (self.users, self.U_full, self.U_loc) if user_side else \
            (self.items, self.V_full, self.V_loc)
        F = torch.as_tensor(F).to(self.device, torch.float32)
        pad = side.padded(torch.arange(side.n, device=self.device)).long()
        full[pad, :self.rank] = F
        loc.copy_(full.view(loc.shape[0], self.world, -1, full.shape[1])[:, self.proc])
        self._dense_cache = {}
        if user_side:  # the YtY a pipelined user half-sweep formed for the old U
            self._yty_u = None

    def fingerprint(self) -> dict:
        """ALSCore.fingerprint over the ratings of all ranks."""
        bits = torch.zeros(1, dtype=torch.int64, device=self.device)
        for blk in self.user_blocks:
            if blk is not None:
                bits += self.K.block_values(blk).view(torch.int32).long().sum().to(self.device)
        all_reduce_capped(bits, "fingerprint", group=self.group)
        return {"nnz": int(self.nnz), "n_users": int(self.n_users), "n_items": int(self.n_items),
                "rating_bits": int(bits), "item_id_sum": int(self.items.ids().long().sum())}

    def user_factor_ids(self) -> torch.Tensor:
        return self.users.ids()

    def exchange_stats(self, rank: Optional[int] = None) -> dict:
        """Padding of the replicated tables and the all-gather bytes one rank receives
        per ALS iteration (both factor halves), at factor rank `rank` (ld = rank
        rounded to 4)."""
        k = self.rank if rank is None else rank
        ld = (k + 3) // 4 * 4
        W = self.world
        recv = sum((W - 1) * s.rows_per_rank * ld * 4 for s in (self.users, self.items))
        return {"padding_users": self.users.padding, "padding_items": self.items.padding,
                "rows_per_chunk": [self.users.rows_per_chunk, self.items.rows_per_chunk],
                "chunks": [self.users.chunks, self.items.chunks],
                "allgather_recv_bytes_per_iter": recv}

    # ---- serving protocol (engine.ALSCore's), on the replicated factors ----
    def _dense(self, user_side: bool, cache: bool = True) -> torch.Tensor:
        """Dense-order copy [n, ld] of one replicated factor table (cached per fit state
        unless cache=False)."""
        self._drain()
        if user_side in self._dense_cache:
            return self._dense_cache[user_side]
        side, full = (self.users, self.U_full) if user_side else (self.items, self.V_full)
        dense = torch.arange(side.n, device=full.device)
        t = full[side.padded(dense).long()].contiguous()
        if cache:
            self._dense_cache[user_side] = t
        return t

    def _ids(self, x) -> torch.Tensor:
        return torch.as_tensor(x).to(self.device).to(torch.int32)

    def predict(self, users, items) -> torch.Tensor:
        """fp64 <u, v> of this rank's pairs (NaN for unknown ids); no collective."""
        self._drain()
        us, its = self.users, self.items
        return self.K.predict(us.keys(self._ids(users)), its.keys(self._ids(items)),
                              us.padded_map(), its.padded_map(), self.U_full, self.V_full,
                              self.rank)

    def rmse(self, users, items, ratings):
        """computeError over the pairs of ALL ranks: local fused (sse, n), then an
        all_reduce (RecommenderSystem.py:123 reduce, :126 count)."""
        self._drain()
        us, its = self.users, self.items
        r = torch.as_tensor(ratings).to(self.device, torch.float32)
        part = self.K.rmse_partial(us.keys(self._ids(users)), its.keys(self._ids(items)), r,
                                   us.padded_map(), its.padded_map(), self.U_full, self.V_full,
                                   self.rank).to(torch.float64)
        all_reduce_capped(part, "rmse partial", group=self.group)
        sse, n = part.tolist()
        return (math.sqrt(sse / n) if n > 0 else float("nan")), int(n)

    def recommend_all(self, top: int, user_side: bool = True):
        """recommendForAll for THIS rank's rows of one side (its partition), against
        the replicated other side: (keys, ids [m, t], scores [m, t]); no collective."""
        side, loc = (self.users, self.U_loc) if user_side else (self.items, self.V_loc)
        other = self.items if user_side else self.users
        Vd = self._dense(not user_side)
        t = min(int(top), other.n)
        keys, ids, scs = [], [], []
        cs = side.cstarts[self.proc]
        oids = other.ids()
        for c in range(side.chunks):
            a, b = int(cs[c]), int(cs[c + 1])
            if b <= a:
                continue
            idx, sc = self.K.topk(loc[c], b - a, Vd, other.n, self.rank, top)
            keys.append(side.ids()[a:b])
            ids.append(oids[idx[:, :t].long().clamp(min=0)])  # empty slots: score -inf
            scs.append(sc[:, :t])
        if not keys:
            e = torch.empty((0, t), device=self.device)
            return torch.empty(0, dtype=torch.int32, device=self.device), e.int(), e
        return torch.cat(keys), torch.cat(ids), torch.cat(scs)

    def recommend_subset(self, ids, top: int, user_side: bool = True):
        side = self.users if user_side else self.items
        other = self.items if user_side else self.users
        keys = torch.unique(self._ids(ids))
        k = side.keys(keys)
        rows = torch.full_like(k, -1, dtype=torch.long)
        ok = k >= 0
        rows[ok] = side.dense_map[k[ok].long()].long()
        keys, rows = keys[rows >= 0], rows[rows >= 0]
        t = min(int(top), other.n)
        if keys.numel() == 0:
            e = torch.empty((0, t), device=self.device)
            return keys, e.int(), e
        Q = self._dense(user_side).index_select(0, rows).contiguous()
        idx, sc = self.K.topk(Q, keys.numel(), self._dense(not user_side), other.n, self.rank,
                              top)
        return keys, other.ids()[idx[:, :t].long().clamp(min=0)], sc[:, :t]

    def recommend_users(self, top: int):
        _, ids, sc = self.recommend_all(top, True)
        return ids, sc

    def recommend_items(self, top: int):
        _, ids, sc = self.recommend_all(top, False)
        return ids, sc

    # ---- factor views in dense order (replicated on every rank) ----
    def user_factors(self, cache: bool = True):
        return self.users.ids(), self._dense(True, cache)[:, :self.rank]

    def item_factors(self, cache: bool = True):
        return self.items.ids(), self._dense(False, cache)[:, :self.rank]
