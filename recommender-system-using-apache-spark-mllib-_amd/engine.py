"""Device-resident ALS engine (one process per GPU).

This is the host side of the hot path that replaces Spark's
``ml.recommendation.ALS.train`` (upstream) as reached from
RecommenderSystem.py:148-149 / :163 / :218, and ``predictAll`` +
``computeError`` (RecommenderSystem.py:103-129, :150, :165, :222, :232).
Every arithmetic step runs in libals_hip.so (HIP, gfx950); torch supplies
device memory, streams and the RNG for the initial factors only.

Data layout in HBM (DESIGN.md "Data layout"):
  users/items id maps  int32[id_space]   (id -> dense row or -1)
  user side  CSR       row_ptr int64[n_u+1], col int32[nnz] (dense item), val f32[nnz]
  item side  CSR       row_ptr int64[n_i+1], col int32[nnz] (dense user), val f32[nnz]
  factors              U f32[n_u, ld], V f32[n_i, ld], ld = roundup(rank, 4), pad cols 0
  schedule per side    light rows (LPT order), heavy rows, chunk tasks
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr

DEFAULT_CHUNK = 4096  # ratings per heavy-row task (round 5: profiles/r05/ab_chunk*.jsonl)


def chunk_for(rank: int, implicit: bool) -> int:
    """Heavy-row task length of a half-sweep (ALSCore's default): a task's fp32 partial
    slot grows as k^2, so explicit fits at rank > 64 take four times the ratings per slot.
    Measured round 5 (profiles/r05/ab_chunk2.jsonl, ab_chunk3.jsonl): configs[3] (k = 128,
    explicit) 4096 / 8192 / 16384 ratings 275.1 / 270.6 / 266.3 ms/iter; at configs[1]
    (k = 64) 8192 took the longest rows' error to 1.2e-6 and at configs[2] (implicit) the
    >2048-rating rows sit at 8e-7 with 4096 already, so those keep 4096."""
    return 4 * DEFAULT_CHUNK if (rank > 64 and not implicit) else DEFAULT_CHUNK
MAX_RANK = 128       # k <= 64: gram_solve_kernel; 64 < k <= 128: W1 (one wavefront per system)
DUAL_MAX_RATINGS = 96  # explicit, 64 < k <= 128: rows this short go through the n x n dual
# (round 5, configs[3]: limit 64 / 80 / 96 -> 288.9 / 275.8 / 267.2 ms/iter, profiles/r05/ab_dual_limit.jsonl)
DUAL_MAX_RATINGS_64 = 32  # explicit, 32 < k <= 64: the same for rows this short

# als_solve_half phase bits (include/als_hip.h ALS_PHASE_*)
PHASE_LAUNCH1, PHASE_LAUNCH2, PHASE_PREP, PHASE_RSCALE, PHASE_DUAL, PHASE_RESCUE = 1, 2, 4, 8, 16, 32
PHASE_ALL = 63


def dual_limit(rank: int) -> int:
    """Longest row (ratings) solved through the n x n dual system at this rank; 0 = none.
    The dual system Y_S Y_S^T + lambda n I is full rank only while n <= rank: a longer
    row would trade the full-rank k x k primal for a rank-deficient n x n system whose
    smallest eigenvalues are lambda n (fp32 error growing as lambda shrinks), so the
    limit is min(96, rank) above rank 64 and 32 (< rank) at ranks 33-64."""
    if rank > 64:
        return min(DUAL_MAX_RATINGS, rank)
    return DUAL_MAX_RATINGS_64 if rank > 32 else 0


def ld_for(rank: int) -> int:
    return (rank + 3) // 4 * 4


class Workspace:
    """One growable device scratch buffer; the library never allocates on a compute call.

    shared_rating_scale: every block solved with this workspace has the same ratings
    (ALSCore's user- and item-major CSR of one rating set), so the rating scale word
    that als_solve_half's phase 8 leaves at the start of the buffer stays valid until
    another call uses the buffer or it is reallocated; solve_half then skips phase 8."""

    def __init__(self, device, shared_rating_scale: bool = False):
        self.device = device
        self.buf: Optional[torch.Tensor] = None
        self.shared_rating_scale = shared_rating_scale
        self.rating_scale_key = None

    def get(self, nbytes: int, keep_scale: bool = False) -> torch.Tensor:
        nbytes = max(int(nbytes), 256)
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            # the scale / rescue-count words: a call without PREP on a fresh buffer
            # must not start from garbage
            self.buf[:256].zero_()
            self.rating_scale_key = None
        if not keep_scale:
            self.rating_scale_key = None
        return self.buf


def _to_device(x, dtype, device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(np.asarray(x)), device=device).to(dtype).contiguous()


# ---------------------------------------------------------------------------
# K1: id maps, CSR, schedule
# ---------------------------------------------------------------------------
@dataclass
class IdIndex:
    """Dense id map of one side (the device form of Spark's sorted InBlock.srcIds).

    Spark accepts any Int id (negative ones included).  The map is indexed by
    `id - offset`; `offset` is the smallest id when ids are negative or the id
    range starts far above 0, else 0 (ids used directly)."""
    map: torch.Tensor       # int32 [id_space], (id - offset) -> dense row or -1
    uniq: torch.Tensor      # int32 [n]   ascending ids - offset
    n: int
    offset: int = 0

    @property
    def id_space(self) -> int:
        return int(self.map.numel())

    def ids(self) -> torch.Tensor:
        """The original ids of the dense rows (ascending), int32."""
        return self.uniq if self.offset == 0 else (self.uniq.long() + self.offset).to(torch.int32)

    def rows_of(self, ids: torch.Tensor) -> torch.Tensor:
        """Dense row (int64) of each id, -1 when unknown."""
        k = ids.long() - self.offset
        ok = (k >= 0) & (k < self.id_space)
        out = torch.full_like(k, -1)
        out[ok] = self.map[k[ok]].long()
        return out

    def keys(self, ids: torch.Tensor) -> torch.Tensor:
        """Query ids -> map keys; ids outside the mapped range -> -1 (unknown)."""
        if self.offset == 0:
            return ids.to(torch.int32).contiguous()
        s = ids.long() - self.offset
        return torch.where((s >= 0) & (s < self.id_space), s, -1).to(torch.int32).contiguous()


MAX_ID_SPACE = 2 ** 31 - 1   # the map is indexed by int32


def id_offset(lo: int, hi: int) -> int:
    """Map offset for ids in [lo, hi]: 0 for the usual non-negative, compact ids."""
    off = 0 if (lo >= 0 and hi < (1 << 26)) else lo
    if hi - off + 1 > MAX_ID_SPACE:
        raise ValueError(f"id range [{lo}, {hi}] spans more than 2^31-1 values; this build "
                         "indexes ids through a dense int32 map")
    return off


def build_index(ids: torch.Tensor, id_space: int, ws: Workspace) -> IdIndex:
    L = _lib.lib()
    dev = ids.device
    mp = torch.empty(id_space, dtype=torch.int32, device=dev)
    uniq = torch.empty(id_space, dtype=torch.int32, device=dev)
    nu = torch.zeros(1, dtype=torch.int32, device=dev)
    need = L.als_index_workspace_bytes(ids.numel(), id_space)
    w = ws.get(need)
    check(L.als_index_build(ptr(ids), ids.numel(), id_space, ptr(mp), ptr(uniq), ptr(nu), ptr(w),
                            w.numel(), stream_ptr(dev)), "als_index_build")
    n = int(nu.item())
    return IdIndex(mp, uniq[:n].clone(), n)


@dataclass
class RatingBlock:
    """One side's ratings in HBM as CSR plus its half-sweep work schedule."""
    n_rows: int
    nnz: int
    row_ptr: torch.Tensor
    col: torch.Tensor
    val: torch.Tensor
    chunk: int
    n_light: int
    n_heavy: int
    n_chunks: int
    light_rows: torch.Tensor
    heavy_rows: torch.Tensor
    heavy_slot_begin: torch.Tensor
    chunk_row: torch.Tensor
    chunk_begin: torch.Tensor
    chunk_end: torch.Tensor
    # short_counts[d] = light rows with <= d ratings, d = 0..DUAL_MAX_RATINGS (host ints)
    short_counts: tuple = ()
    short_nnz: tuple = ()   # ratings of those rows

    @property
    def n_short(self) -> int:
        return self.short_counts[-1] if self.short_counts else 0

    def n_dual(self, rank: int) -> int:
        """Light rows solved through the n x n dual system at this rank (explicit, reg > 0):
        the tail of the longest-first light list with <= dual_limit(rank) ratings."""
        d = dual_limit(rank)
        return self.short_counts[d] if (d and self.short_counts) else 0

    def dual_nnz(self, rank: int) -> int:
        """Ratings of the dual-path rows at this rank."""
        d = dual_limit(rank)
        return self.short_nnz[d] if (d and self.short_nnz) else 0


def build_block(row_ids: torch.Tensor, row_index: IdIndex, col_ids: torch.Tensor,
                col_index: IdIndex, vals: torch.Tensor, ws: Workspace,
                chunk: int = DEFAULT_CHUNK) -> RatingBlock:
    L = _lib.lib()
    dev = row_ids.device
    nnz = int(row_ids.numel())
    n_rows = row_index.n
    row_ptr = torch.empty(n_rows + 1, dtype=torch.int64, device=dev)
    col = torch.empty(nnz, dtype=torch.int32, device=dev)
    val = torch.empty(nnz, dtype=torch.float32, device=dev)
    w = ws.get(L.als_csr_workspace_bytes(nnz, n_rows))
    check(L.als_csr_build(ptr(row_ids), ptr(row_index.map), ptr(col_ids), ptr(col_index.map),
                          ptr(vals), nnz, n_rows, ptr(row_ptr), ptr(col), ptr(val), ptr(w),
                          w.numel(), stream_ptr(dev)), "als_csr_build")
    return schedule_block(n_rows, nnz, row_ptr, col, val, ws, chunk)


def schedule_block(n_rows, nnz, row_ptr, col, val, ws: Workspace, chunk: int = DEFAULT_CHUNK
                   ) -> RatingBlock:
    L = _lib.lib()
    dev = row_ptr.device
    counts = torch.zeros(3, dtype=torch.int32, device=dev)
    check(L.als_schedule_count(ptr(row_ptr), n_rows, chunk, ptr(counts), stream_ptr(dev)),
          "als_schedule_count")
    n_light, n_heavy, n_chunks = (int(x) for x in counts.tolist())
    i32 = dict(dtype=torch.int32, device=dev)
    light = torch.empty(max(n_light, 1), **i32)
    heavy = torch.empty(max(n_heavy, 1), **i32)
    slot_begin = torch.empty(n_heavy + 1, **i32)
    crow = torch.empty(max(n_chunks, 1), **i32)
    cbeg = torch.empty(max(n_chunks, 1), dtype=torch.int64, device=dev)
    cend = torch.empty(max(n_chunks, 1), dtype=torch.int64, device=dev)
    w = ws.get(L.als_schedule_workspace_bytes(n_rows))
    check(L.als_schedule_build(ptr(row_ptr), n_rows, chunk, n_light, n_heavy, n_chunks,
                               ptr(light), ptr(heavy), ptr(slot_begin), ptr(crow), ptr(cbeg),
                               ptr(cend), ptr(w), w.numel(), stream_ptr(dev)),
          "als_schedule_build")
    counts, nzs = (0,) * (DUAL_MAX_RATINGS + 1), (0,) * (DUAL_MAX_RATINGS + 1)
    if n_light > 0:  # light rows are ordered by decreasing degree: the short ones are last
        lr = light[:n_light].long()
        deg = row_ptr[lr + 1] - row_ptr[lr]
        short = deg[deg <= DUAL_MAX_RATINGS]
        h = torch.bincount(short, minlength=DUAL_MAX_RATINGS + 1).to(torch.int64)
        w = h * torch.arange(DUAL_MAX_RATINGS + 1, device=h.device)
        counts = tuple(int(x) for x in torch.cumsum(h, 0).tolist())
        nzs = tuple(int(x) for x in torch.cumsum(w, 0).tolist())
    return RatingBlock(n_rows, nnz, row_ptr, col, val, chunk, n_light, n_heavy, n_chunks, light,
                       heavy, slot_begin, crow, cbeg, cend, counts, nzs)


# ---------------------------------------------------------------------------
# K2/K3/K2b
# ---------------------------------------------------------------------------
def k_pad(rank: int) -> int:
    return int(_lib.lib().als_k_pad(rank))


def compute_yty(Y: torch.Tensor, n: int, rank: int, ws: Workspace) -> torch.Tensor:
    """fp64 YtY (lower-packed, k_pad) of the first n rows of Y."""
    L = _lib.lib()
    kp = k_pad(rank)
    out = torch.empty(kp * (kp + 1) // 2, dtype=torch.float64, device=Y.device)
    w = ws.get(L.als_yty_workspace_bytes(n, rank))
    check(L.als_yty(ptr(Y), n, Y.shape[1], rank, ptr(out), ptr(w), w.numel(),
                    stream_ptr(Y.device)), "als_yty")
    return out


def solve_half(block: RatingBlock, Y: torch.Tensor, X: torch.Tensor, rank: int, reg: float,
               implicit: bool, alpha: float, yty: Optional[torch.Tensor],
               status: torch.Tensor, ws: Workspace, phases: int = PHASE_ALL,
               ws_chunks: Optional[int] = None, dual: bool = True,
               ws_rows: Optional[int] = None) -> None:
    """One computeFactors pass: X[row] <- solve(A_row, b_row) for every row of `block`.
    phases (PHASE_* bits, als_hip.h ALS_PHASE_*): PREP (max |Y|, split table), RSCALE
    (rating scale), LAUNCH1 (chunk partials + primal light rows), DUAL (dual-path light
    rows), LAUNCH2 (heavy rows), RESCUE (rows outside the split window); PHASE_ALL = all
    in order.  ws_chunks / ws_rows: size the workspace for this many heavy-row chunks /
    rows (blocks sharing one Y prep).
    dual: explicit, reg > 0 — rows with <= dual_limit(rank) ratings are solved through
    the equivalent n x n dual system (als_hip.h n_light_primal); False keeps every row
    on the k x k normal equations."""
    L = _lib.lib()
    use_dual = dual and not implicit and reg > 0
    n_primal = block.n_light - block.n_dual(rank) if use_dual else block.n_light
    n_rows = max(block.n_light + block.n_heavy, ws_rows or 0)
    w = ws.get(L.als_solve_workspace_bytes(rank, max(block.n_chunks, ws_chunks or 0), Y.shape[0],
                                           n_rows), keep_scale=True)
    key = (w.data_ptr(), w.numel())
    if (phases & PHASE_RSCALE) and ws.shared_rating_scale and ws.rating_scale_key == key:
        phases &= ~PHASE_RSCALE  # the rating scale word of this rating set is already in place
        if phases == 0:
            return
    check(L.als_solve_half(ptr(block.row_ptr), ptr(block.col), ptr(block.val),
                           ptr(block.light_rows), block.n_light, n_primal,
                           ptr(block.heavy_rows),
                           ptr(block.heavy_slot_begin), block.n_heavy, ptr(block.chunk_row),
                           ptr(block.chunk_begin), ptr(block.chunk_end), block.n_chunks, 0, 0,
                           ptr(Y), Y.shape[0], ptr(X), X.shape[1], rank, float(reg),
                           int(bool(implicit)),
                           float(alpha), ptr(yty), ptr(status), ptr(w), w.numel(), int(phases),
                           stream_ptr(X.device)), "als_solve_half")
    if (phases & PHASE_RSCALE) and ws.shared_rating_scale:
        ws.rating_scale_key = key


@dataclass
class SplitSchedule:
    """Two-segment schedule of one CSR block (ABI 6, the sharded engine's pipelined item
    half-sweep).  Row r's ratings are [row_ptr[r], seg[r]) — the early segment, whose
    source rows lie in the first n_src_early rows of Y (already gathered) — then
    [seg[r], row_ptr[r+1]) (the late segment: the source chunk still arriving).  Each
    segment is cut into <= chunk-rating tasks; every row goes through the heavy-row
    path (fp32 task partials summed per row in fp64, then solved), early slots first.
    Slots are numbered from slot_base (several blocks sharing one workspace and one Y
    prep keep disjoint slot ranges: ShardedALS's item chunks)."""
    n_src_early: int
    rows: torch.Tensor          # int32 [n]: every row of the block, ascending
    slot_begin: torch.Tensor    # int32 [n+1]: early slots of row r
    slot_begin2: torch.Tensor   # int32 [n+1]: late slots of row r (after all early ones)
    early: tuple                # (chunk_row, chunk_begin, chunk_end, n_tasks)
    late: tuple
    slot_base: int = 0          # first slot of this block's range in the workspace

    @property
    def n_slots(self) -> int:
        """Slots of the workspace up to this block's last (slot_base included)."""
        return self.slot_base + self.early[3] + self.late[3]


def _segment_tasks(row_ids, begin, end, chunk: int, dev):
    """<= chunk-rating tasks over the per-row ranges [begin[r], end[r])."""
    ln = (end - begin).clamp(min=0)
    cnt = (ln + chunk - 1) // chunk
    n = int(cnt.sum())
    slot_begin = torch.zeros(len(ln) + 1, dtype=torch.int64, device=dev)
    slot_begin[1:] = torch.cumsum(cnt, 0)
    if n == 0:
        z32, z64 = torch.zeros(1, dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int64,
                                                                              device=dev)
        return slot_begin, (z32, z64, z64, 0)
    crow = torch.repeat_interleave(torch.arange(len(ln), device=dev), cnt)
    j = torch.arange(n, device=dev) - slot_begin[:-1][crow]
    cb = begin[crow] + j * chunk
    ce = torch.minimum(cb + chunk, end[crow])
    return slot_begin, (row_ids[crow].to(torch.int32).contiguous(), cb.contiguous(),
                        ce.contiguous(), n)


def split_schedule(block: RatingBlock, seg: torch.Tensor, n_src_early: int,
                   chunk: int = DEFAULT_CHUNK, slot_base: int = 0) -> SplitSchedule:
    """The two-segment schedule of `block` (its rows' ratings ordered early-first, seg[r]
    = end of row r's early segment), its slots numbered from slot_base."""
    dev = block.row_ptr.device
    n = block.n_rows
    rp = block.row_ptr
    seg = seg.to(dev, torch.int64)
    rows = torch.arange(max(n, 1), dtype=torch.int32, device=dev)
    sb1, early = _segment_tasks(rows[:n], rp[:-1], seg, chunk, dev)
    sb2, late = _segment_tasks(rows[:n], seg, rp[1:], chunk, dev)
    sb1 = sb1 + slot_base
    sb2 = sb2 + early[3] + slot_base
    return SplitSchedule(int(n_src_early), rows, sb1.to(torch.int32).contiguous(),
                         sb2.to(torch.int32).contiguous(), early, late, int(slot_base))


def solve_half_split(block: RatingBlock, sched: SplitSchedule, part: str, Y: torch.Tensor,
                     X: torch.Tensor, rank: int, reg: float, implicit: bool, alpha: float,
                     yty: Optional[torch.Tensor], status: torch.Tensor, ws: Workspace,
                     prep: bool = True, ws_slots: Optional[int] = None,
                     ws_rows: Optional[int] = None) -> None:
    """One half of a two-segment half-sweep (ABI 6).  part "early": the early segments'
    task partials from the first sched.n_src_early rows of Y (PREP over that prefix,
    RSCALE, LAUNCH1), while the rest of Y may still be arriving; "late": the late
    segments' partials from all of Y, then every row's slots summed and solved
    (LAUNCH2) and the rescue (RESCUE, over the row's full ratings).  Both calls on
    the same workspace, early first, in stream order.  Both pass slot_begin2 (it marks
    the schedule two-segment: no heavy row is solved before its late partials).
    prep=False: Y's prep for this part was done by an earlier call on this workspace
    (blocks sharing one workspace with disjoint slot ranges, sized by ws_slots /
    ws_rows for the largest: all early calls first, then all late ones)."""
    L = _lib.lib()
    n = block.n_rows
    w = ws.get(L.als_solve_workspace_bytes(rank, max(sched.n_slots, ws_slots or 0), Y.shape[0],
                                           max(n, ws_rows or 0)))
    if part == "early":
        crow, cb, ce, nt = sched.early
        ph, slot0, n_src = PHASE_PREP | PHASE_RSCALE | PHASE_LAUNCH1, sched.slot_base, sched.n_src_early
    elif part == "late":
        crow, cb, ce, nt = sched.late
        ph = PHASE_PREP | PHASE_RSCALE | PHASE_LAUNCH1 | PHASE_LAUNCH2 | PHASE_RESCUE
        slot0, n_src = sched.slot_base + sched.early[3], Y.shape[0]
    else:
        raise ValueError(f"part must be 'early' or 'late', got {part!r}")
    if not prep:
        ph &= ~PHASE_PREP
    sb2 = sched.slot_begin2
    check(L.als_solve_half(ptr(block.row_ptr), ptr(block.col), ptr(block.val),
                           ptr(block.light_rows), 0, 0, ptr(sched.rows), ptr(sched.slot_begin), n,
                           ptr(crow), ptr(cb), ptr(ce), nt, ptr(sb2), slot0,
                           ptr(Y), n_src, ptr(X), X.shape[1], rank, float(reg),
                           int(bool(implicit)), float(alpha), ptr(yty), ptr(status), ptr(w),
                           w.numel(), int(ph), stream_ptr(X.device)), "als_solve_half (split)")


def raise_status(s: int, where: str = "") -> None:
    """Raise for a non-zero solve status word: row + 1 of a failed Cholesky (Spark's
    dppsv info > 0), or -1 when the fp64 rescue list overflowed (als_solve_half's
    LAUNCH phases ran twice without the RESCUE phase between them)."""
    if s < 0:
        raise RuntimeError(f"als_solve_half rescue list overflow{where}: the LAUNCH phases ran "
                           "again before the RESCUE phase consumed the list (unsolved rows)")
    if s > 0:
        raise RuntimeError(
            f"Cholesky failed (non-positive pivot) for dense row {s - 1}{where}: the normal "
            "equations are not positive definite (Spark raises from LAPACK dppsv here)")


# ---------------------------------------------------------------------------
# K4/K5
# ---------------------------------------------------------------------------
def predict_pairs(u: torch.Tensor, i: torch.Tensor, uidx: IdIndex, iidx: IdIndex,
                  U: torch.Tensor, V: torch.Tensor, rank: int) -> torch.Tensor:
    L = _lib.lib()
    u, i = uidx.keys(u), iidx.keys(i)
    out = torch.empty(u.numel(), dtype=torch.float64, device=U.device)
    check(L.als_predict(ptr(u), ptr(i), u.numel(), ptr(uidx.map), uidx.id_space, ptr(iidx.map),
                        iidx.id_space, ptr(U), ptr(V), U.shape[1], rank, ptr(out),
                        stream_ptr(U.device)), "als_predict")
    return out


def rmse_pairs(u, i, r, uidx: IdIndex, iidx: IdIndex, U, V, rank: int, ws: Workspace):
    """(sse, count) over pairs with both ids known (computeError's join)."""
    L = _lib.lib()
    u, i = uidx.keys(u), iidx.keys(i)
    out = torch.empty(2, dtype=torch.float64, device=U.device)
    w = ws.get(L.als_rmse_workspace_bytes(u.numel()))
    check(L.als_rmse_partial(ptr(u), ptr(i), ptr(r), u.numel(), ptr(uidx.map), uidx.id_space,
                             ptr(iidx.map), iidx.id_space, ptr(U), ptr(V), U.shape[1], rank,
                             ptr(out), ptr(w), w.numel(), stream_ptr(U.device)),
          "als_rmse_partial")
    return out


def ids_of(ids: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """Ids of top-k dense rows.  A slot the kernel left empty (idx -1, score -inf: every
    score of that query row NaN, from non-finite factors) keeps a placeholder id; the
    callers drop slots whose score is not finite (valid_slots)."""
    return ids[idx.long().clamp(min=0)]


def topk_rows(Q: torch.Tensor, n_q: int, V: torch.Tensor, n_v: int, rank: int, top: int):
    """(idx int32 [n_q, top], score f32 [n_q, top]); idx = dense V row, -1 past n_v."""
    L = _lib.lib()
    idx = torch.empty((n_q, top), dtype=torch.int32, device=Q.device)
    sc = torch.empty((n_q, top), dtype=torch.float32, device=Q.device)
    w = torch.empty(int(L.als_topk_workspace_bytes(n_q, n_v, rank, top)), dtype=torch.uint8,
                    device=Q.device)
    check(L.als_topk(ptr(Q), n_q, ptr(V), n_v, Q.shape[1], rank, top, ptr(idx), ptr(sc), ptr(w),
                     w.numel(), stream_ptr(Q.device)), "als_topk")
    return idx, sc


# ---------------------------------------------------------------------------
# The engine
# ---------------------------------------------------------------------------
def make_engine(users, items, ratings, device=None):
    """The engine behind ALS.fit / ALS.train: one GPU (ALSCore), or — when this process
    is one rank of an initialised torch.distributed group of world size > 1 —
    the sharded engine (distributed.ShardedALS), fed with this rank's partition
    of the ratings (the role of a Spark DataFrame partition)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        from .distributed import ShardedALS
        return ShardedALS(users, items, ratings, device=device)
    return ALSCore(users, items, ratings, device=device)


class ALSCore:
    """Ratings, id maps, both CSR sides and both factor matrices resident on one GPU."""

    def __init__(self, users, items, ratings, device=None, chunk: Optional[int] = None):
        """chunk: ratings per heavy-row task; None = chunk_for(rank, implicit) of each
        half-sweep (the blocks are rescheduled when a fit asks for another length)."""
        _lib.require_gpu()
        self._auto_chunk = chunk is None
        chunk = DEFAULT_CHUNK if chunk is None else chunk
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        # both CSR sides hold the same ratings: one rating scale for every half-sweep
        self.ws = Workspace(self.device, shared_rating_scale=True)
        # computeYtY's task slots in a buffer of their own: written over the solve
        # workspace they would clobber its rating scale word, re-measured every half-sweep
        self.ws_yty = Workspace(self.device)
        u = _to_device(users, torch.int32, self.device)
        i = _to_device(items, torch.int32, self.device)
        r = _to_device(ratings, torch.float32, self.device)
        if not (u.numel() == i.numel() == r.numel()):
            raise ValueError("users, items and ratings must have the same length")
        if u.numel() == 0:
            raise ValueError("ALS needs at least one rating")
        umin, umax = int(u.min()), int(u.max())
        imin, imax = int(i.min()), int(i.max())
        uoff, ioff = id_offset(umin, umax), id_offset(imin, imax)
        if uoff:
            u = (u.long() - uoff).to(torch.int32)
        if ioff:
            i = (i.long() - ioff).to(torch.int32)
        self.nnz = int(u.numel())
        self.uidx = build_index(u, umax - uoff + 1, self.ws)
        self.iidx = build_index(i, imax - ioff + 1, self.ws)
        self.uidx.offset, self.iidx.offset = uoff, ioff
        self.user_block = build_block(u, self.uidx, i, self.iidx, r, self.ws, chunk)
        self.item_block = build_block(i, self.iidx, u, self.uidx, r, self.ws, chunk)
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.U: Optional[torch.Tensor] = None
        self.V: Optional[torch.Tensor] = None
        self.rank = 0

    @classmethod
    def from_factors(cls, user_ids, U, item_ids, V, device=None) -> "ALSCore":
        """A serving-only core (no ratings, cannot fit) from saved factors: ids ascending,
        U/V host or device arrays [n, rank].  predict / rmse / top-k run as after fit()."""
        _lib.require_gpu()
        self = cls.__new__(cls)
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.ws = Workspace(self.device)
        self.ws_yty = self.ws
        self.nnz = 0
        self._auto_chunk = False
        self.user_block = self.item_block = None
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        U = _to_device(U, torch.float32, self.device)
        V = _to_device(V, torch.float32, self.device)
        rank = int(U.shape[1])
        if V.shape[1] != rank or not (1 <= rank <= MAX_RANK):
            raise ValueError(f"factor ranks {U.shape[1]}/{V.shape[1]} invalid (max {MAX_RANK})")
        idx = []
        for ids, F in ((user_ids, U), (item_ids, V)):
            ids = _to_device(ids, torch.int32, self.device)
            if ids.numel() != F.shape[0] or ids.numel() == 0:
                raise ValueError("factor ids must be non-empty and match the rows")
            if ids.numel() > 1 and not bool((ids[1:] > ids[:-1]).all()):
                raise ValueError("factor ids must be strictly ascending")
            off = id_offset(int(ids.min()), int(ids.max()))
            key = (ids.long() - off)
            mp = torch.full((int(key.max()) + 1,), -1, dtype=torch.int32, device=self.device)
            mp[key] = torch.arange(ids.numel(), dtype=torch.int32, device=self.device)
            idx.append(IdIndex(mp, key.to(torch.int32), int(ids.numel()), off))
        self.uidx, self.iidx = idx
        self.rank = rank
        ld = ld_for(rank)
        self.U = torch.zeros((U.shape[0], ld), dtype=torch.float32, device=self.device)
        self.V = torch.zeros((V.shape[0], ld), dtype=torch.float32, device=self.device)
        self.U[:, :rank] = U
        self.V[:, :rank] = V
        return self

    @property
    def n_users(self) -> int:
        return self.uidx.n

    @property
    def n_items(self) -> int:
        return self.iidx.n

    # Spark ALS.initialize: unit-norm Gaussian rows, fp32.
    def init_factors(self, rank: int, seed: int = 0, U0=None) -> None:
        if rank < 1 or rank > MAX_RANK:
            raise ValueError(f"rank must be in [1, {MAX_RANK}] on this build, got {rank}")
        self.rank = rank
        ld = ld_for(rank)
        self.U = torch.zeros((self.n_users, ld), dtype=torch.float32, device=self.device)
        self.V = torch.zeros((self.n_items, ld), dtype=torch.float32, device=self.device)
        if U0 is not None:
            U0 = _to_device(U0, torch.float32, self.device)
            if tuple(U0.shape) != (self.n_users, rank):
                raise ValueError(f"U0 must have shape {(self.n_users, rank)}")
            self.U[:, :rank] = U0
        else:
            g = torch.Generator(device=self.device)
            g.manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
            x = torch.randn((self.n_users, rank), generator=g, device=self.device,
                            dtype=torch.float32)
            self.U[:, :rank] = x / torch.linalg.vector_norm(x, dim=1, keepdim=True)

    def schedule_for(self, implicit: bool) -> None:
        """The default heavy-row task length for this fit's rank and feedback type (no-op
        when the core was built with an explicit chunk)."""
        if self._auto_chunk:
            self.rechunk(chunk_for(self.rank, implicit))

    def rechunk(self, chunk: int) -> None:
        """Reschedule both sides for `chunk`-rating heavy-row tasks (same CSR)."""
        for name in ("user_block", "item_block"):
            b = getattr(self, name)
            if b.chunk != chunk:
                setattr(self, name, schedule_block(b.n_rows, b.nnz, b.row_ptr, b.col, b.val,
                                                   self.ws, chunk))

    def half_sweep_items(self, reg, implicit=False, alpha=1.0):
        self.schedule_for(implicit)
        yty = compute_yty(self.U, self.n_users, self.rank, self.ws_yty) if implicit else None
        solve_half(self.item_block, self.U, self.V, self.rank, reg, implicit, alpha, yty,
                   self.status, self.ws)

    def half_sweep_users(self, reg, implicit=False, alpha=1.0):
        self.schedule_for(implicit)
        yty = compute_yty(self.V, self.n_items, self.rank, self.ws_yty) if implicit else None
        solve_half(self.user_block, self.V, self.U, self.rank, reg, implicit, alpha, yty,
                   self.status, self.ws)

    def iterate(self, reg, implicit=False, alpha=1.0):
        """One ALS iteration in Spark's order: items from users, then users from items."""
        self.half_sweep_items(reg, implicit, alpha)
        self.half_sweep_users(reg, implicit, alpha)

    def check_status(self) -> None:
        raise_status(int(self.status.item()))

    def fit(self, rank, max_iter, reg, implicit=False, alpha=1.0, seed=0, U0=None,
            checkpoint_dir=None, checkpoint_interval=10, resume=False):
        """max_iter ALS iterations from the seeded (or given U0) start.  checkpoint_dir:
        write U, V every checkpoint_interval iterations (checkpoint.py); resume
        (True / "auto"): continue from the checkpoint there at its iteration."""
        from . import checkpoint as C
        init = C.init_key(seed, U0) if checkpoint_dir else None
        start, Uc, Vc = C.resume_point(checkpoint_dir, resume, self, rank, reg, implicit, alpha,
                                       max_iter, init)
        self.init_factors(rank, seed, Uc if Uc is not None else U0)
        if Vc is not None:
            self.V[:, :rank] = _to_device(Vc, torch.float32, self.device)
        self.status.zero_()
        for it in range(start, max_iter):
            self.iterate(reg, implicit, alpha)
            C.maybe_save(checkpoint_dir, checkpoint_interval, it + 1, self, rank, reg, implicit,
                         alpha, init=init)
        self.check_status()
        return self

    def fingerprint(self) -> dict:
        """Order-independent identity of the training ratings (checkpoint matching)."""
        v = self.user_block.val
        return {"nnz": int(self.nnz), "n_users": int(self.n_users), "n_items": int(self.n_items),
                "rating_bits": int(v.view(torch.int32).long().sum()),
                "item_id_sum": int(self.iidx.ids().long().sum())}

    def user_factor_ids(self) -> torch.Tensor:
        return self.uidx.ids()

    # ---- K4 / K5 (the serving protocol shared with distributed.ShardedALS) ----
    def predict(self, users, items) -> torch.Tensor:
        """fp64 <u, v> per pair (MatrixFactorizationModel.predict's ddot); NaN where
        either id is unknown."""
        u = _to_device(users, torch.int32, self.device)
        i = _to_device(items, torch.int32, self.device)
        return predict_pairs(u, i, self.uidx, self.iidx, self.U, self.V, self.rank)

    def rmse(self, users, items, ratings):
        """(sqrt(sum (r - p)^2 / n), n) over the pairs whose ids are both known —
        computeError (RecommenderSystem.py:103-129) fused into one pass."""
        u = _to_device(users, torch.int32, self.device)
        i = _to_device(items, torch.int32, self.device)
        r = _to_device(ratings, torch.float32, self.device)
        sse, n = rmse_pairs(u, i, r, self.uidx, self.iidx, self.U, self.V, self.rank,
                            self.ws).tolist()
        return (math.sqrt(sse / n) if n > 0 else float("nan")), int(n)

    def _sides(self, user_side: bool):
        if user_side:
            return self.uidx, self.U, self.iidx, self.V
        return self.iidx, self.V, self.uidx, self.U

    def recommend_all(self, top: int, user_side: bool = True):
        """recommendForAll: for every row of one side (dense order) its `top` best
        rows of the other side.  Returns (keys [n], ids [n, t], scores [n, t]) on the
        device, t = min(top, rows of the other side), scores descending."""
        qi, Q, oi, Vo = self._sides(user_side)
        idx, sc = topk_rows(Q, qi.n, Vo, oi.n, self.rank, top)
        t = min(int(top), oi.n)
        return qi.ids(), ids_of(oi.ids(), idx[:, :t]), sc[:, :t]

    def recommend_subset(self, ids, top: int, user_side: bool = True):
        """recommendForUserSubset / ForItemSubset: distinct known ids of `ids`
        (ascending) -> (keys, ids [m, t], scores [m, t])."""
        qi, Q, oi, Vo = self._sides(user_side)
        q = _to_device(ids, torch.int32, self.device)
        keys = torch.unique(q)
        rows = qi.rows_of(keys)
        known = rows >= 0
        keys, rows = keys[known], rows[known]
        t = min(int(top), oi.n)
        if keys.numel() == 0:
            return keys, torch.empty((0, t), dtype=torch.int32, device=self.device), \
                torch.empty((0, t), dtype=torch.float32, device=self.device)
        Qs = Q.index_select(0, rows.long()).contiguous()
        idx, sc = topk_rows(Qs, keys.numel(), Vo, oi.n, self.rank, top)
        return keys, ids_of(oi.ids(), idx[:, :t]), sc[:, :t]

    def recommend_users(self, top: int):
        """For every user (dense order): top items as (item ids, scores)."""
        _, ids, sc = self.recommend_all(top, True)
        return ids, sc

    def recommend_items(self, top: int):
        _, ids, sc = self.recommend_all(top, False)
        return ids, sc

    def user_factors(self, cache: bool = True):
        return self.uidx.ids(), self.U[:, :self.rank]

    def item_factors(self, cache: bool = True):
        return self.iidx.ids(), self.V[:, :self.rank]
