"""Factor checkpoints and resume at a half-sweep boundary.

Spark's ALS (ml/recommendation/ALS.scala `train`, upstream, not vendored) only
truncates RDD lineage every `checkpointInterval` iterations when a checkpoint dir
is set; the reference never sets one (RecommenderSystem.py has no
setCheckpointDir).  On the GPU there is no lineage, so a checkpoint here is the
state a restarted job needs: the user factors after a completed iteration.  Only
U feeds the next iteration (its item half-sweep reads U; V is recomputed from it,
SURVEY §3A.5), so resuming from U at iteration t and running to T gives the same
factors as an uninterrupted T-iteration fit.

Layout of a checkpoint directory (host formats, nothing pickled):
    als_state.json      {"format": 2, "iteration": t, "generation": "gen-<t>-<tag>",
                         "rank", "regParam", "implicitPrefs", "alpha",
                         "init": {"seed": s} | {"U0": sha1}, "data": fingerprint}
    gen-<t>-<tag>/      one complete generation:
        user_ids.npy        int32 [n_users]   dense order (ascending ids)
        user_factors.npy    float32 [n_users, rank]
        item_ids.npy, item_factors.npy        the same for V (needed only when the
                            checkpoint is already at the requested iteration count:
                            V_t came from U_{t-1}, which is not kept)
A save writes a NEW generation directory (fsynced), then atomically replaces
als_state.json (the commit point), then deletes the older generations.  A job
killed at any point leaves als_state.json naming one complete generation, and
its factors are always those of the iteration the JSON states.

Matching: the ratings fingerprint, rank, regParam, implicitPrefs and alpha must
agree.  In "auto" mode (ALS.fit with a checkpoint dir, Spark's checkpointInterval
semantics: a checkpoint never changes the model) the initialisation must agree
too — a different seed or explicit start is a different fit; resume=True is the
explicit "continue from this checkpoint" and ignores the initialisation.

Multi-process: resume_point_agreed() lets process 0 decide and broadcasts the
decision (and the factors) to every rank, so all ranks start at the same
iteration from the same state even without a shared filesystem.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import uuid
from dataclasses import dataclass
from typing import Optional

import numpy as np

STATE = "als_state.json"
IDS = "user_ids.npy"
FACTORS = "user_factors.npy"
IIDS = "item_ids.npy"
IFACTORS = "item_factors.npy"
FORMAT = 2
_GEN = "gen-"


@dataclass
class State:
    iteration: int
    rank: int
    reg: float
    implicit: bool
    alpha: float
    data: dict
    user_ids: np.ndarray
    U: np.ndarray
    item_ids: np.ndarray
    V: np.ndarray
    init: Optional[dict] = None


def init_key(seed, U0) -> dict:
    """How a fit starts: its seed, or a digest of an explicit initial U."""
    if U0 is not None:
        a = np.ascontiguousarray(np.asarray(
            U0.detach().cpu().numpy() if hasattr(U0, "detach") else U0, dtype=np.float32))
        return {"U0": hashlib.sha1(a.tobytes()).hexdigest() + f":{a.shape}"}
    return {"seed": int(seed)}


def _fsync_file(path: str) -> None:
    with open(path, "rb") as f:
        os.fsync(f.fileno())


def _fsync_dir(path: str) -> None:
    try:
        fd = os.open(path, os.O_RDONLY)
    except OSError:
        return
    try:
        os.fsync(fd)
    except OSError:
        pass
    finally:
        os.close(fd)


def save(dirpath: str, iteration: int, rank: int, reg: float, implicit: bool, alpha: float,
         data: dict, user_ids, U, item_ids, V, init: Optional[dict] = None) -> None:
    """Write the state after `iteration` completed iterations (a new generation, then
    the atomic commit of als_state.json, then removal of the older generations)."""
    os.makedirs(dirpath, exist_ok=True)
    # the layout this commit replaces: a format-1 checkpoint kept its arrays next to
    # the JSON, and only then are same-named top-level files ours to remove
    prev_format = None
    try:
        with open(os.path.join(dirpath, STATE)) as f:
            prev_format = json.load(f).get("format")
    except (OSError, ValueError, AttributeError):
        pass
    gen = f"{_GEN}{int(iteration):06d}-{uuid.uuid4().hex[:8]}"
    tmp = os.path.join(dirpath, "." + gen + ".tmp")
    os.makedirs(tmp)
    for ids_name, f_name, ids, F in ((IDS, FACTORS, user_ids, U), (IIDS, IFACTORS, item_ids, V)):
        ids = np.ascontiguousarray(np.asarray(ids), dtype=np.int32)
        F = np.ascontiguousarray(np.asarray(F), dtype=np.float32)
        if F.shape != (ids.shape[0], rank):
            shutil.rmtree(tmp, ignore_errors=True)
            raise ValueError(f"factor table {F.shape} does not match {ids.shape[0]} ids x rank "
                             f"{rank}")
        for name, arr in ((ids_name, ids), (f_name, F)):
            p = os.path.join(tmp, name)
            np.save(p, arr, allow_pickle=False)
            _fsync_file(p)
    _fsync_dir(tmp)
    os.replace(tmp, os.path.join(dirpath, gen))
    _fsync_dir(dirpath)
    meta = {"format": FORMAT, "iteration": int(iteration), "generation": gen, "rank": int(rank),
            "regParam": float(reg), "implicitPrefs": bool(implicit), "alpha": float(alpha),
            "init": init, "data": data}
    tmpj = os.path.join(dirpath, STATE + ".tmp")
    with open(tmpj, "w") as f:
        json.dump(meta, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmpj, os.path.join(dirpath, STATE))  # the commit point
    _fsync_dir(dirpath)
    for name in os.listdir(dirpath):  # older generations, stale temporaries
        if name != gen and (name.startswith(_GEN) or (name.startswith("." + _GEN)
                                                       and name.endswith(".tmp"))):
            shutil.rmtree(os.path.join(dirpath, name), ignore_errors=True)
    if prev_format == 1:  # the replaced format-1 layout's top-level arrays
        for name in (IDS, FACTORS, IIDS, IFACTORS):
            try:
                os.remove(os.path.join(dirpath, name))
            except FileNotFoundError:
                pass


def load(dirpath: str) -> Optional[State]:
    """The checkpoint in `dirpath`, or None when there is none."""
    p = os.path.join(dirpath, STATE)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        m = json.load(f)
    fmt = m.get("format")
    if fmt == 2:
        base = os.path.join(dirpath, m["generation"])
    elif fmt == 1:  # round-2 layout: files next to the JSON
        base = dirpath
    else:
        raise ValueError(f"{p}: unknown checkpoint format {fmt}")
    arr = [np.load(os.path.join(base, n), allow_pickle=False)
           for n in (IDS, FACTORS, IIDS, IFACTORS)]
    return State(int(m["iteration"]), int(m["rank"]), float(m["regParam"]),
                 bool(m["implicitPrefs"]), float(m["alpha"]), m["data"], *arr,
                 init=m.get("init"))


def mismatch(st: State, rank: int, reg: float, implicit: bool, alpha: float, data: dict,
             user_ids, init: Optional[dict] = None) -> Optional[str]:
    """Why `st` cannot seed this fit (None when it can).  init: compare the
    initialisation too (auto mode)."""
    if st.rank != rank:
        return f"rank {st.rank} != {rank}"
    if st.reg != float(reg) or st.implicit != bool(implicit) or \
            (implicit and st.alpha != float(alpha)):
        return "regParam / implicitPrefs / alpha differ"
    if st.data != data:
        return f"ratings differ (checkpoint {st.data}, now {data})"
    ids = np.asarray(user_ids, dtype=np.int32)
    if st.user_ids.shape != ids.shape or not np.array_equal(st.user_ids, ids):
        return "user ids differ"
    if st.U.shape != (ids.shape[0], rank):
        return f"factor table shape {st.U.shape}"
    if init is not None and st.init != init:
        return f"initialisation differs (checkpoint {st.init}, now {init})"
    return None


def resume_point(dirpath: Optional[str], resume, engine, rank: int, reg: float, implicit: bool,
                 alpha: float, max_iter: int, init: Optional[dict] = None,
                 fingerprint: Optional[dict] = None):
    """(start iteration, U0, V0) for engine.fit; U0/V0 None for a fresh start, V0 set
    only when the checkpoint is already at max_iter.  resume: False = start fresh;
    True = the checkpoint must exist and match (ValueError otherwise; the
    initialisation is not compared); "auto" = use it when it matches, initialisation
    included, else start fresh.  fingerprint: the engine's (precomputed by every
    rank of a sharded engine, where it is a collective)."""
    if not resume or not dirpath:
        return 0, None, None
    st = load(dirpath)
    if st is None:
        if resume is True:
            raise ValueError(f"no ALS checkpoint in {dirpath}")
        return 0, None, None
    ids = engine.user_factor_ids().cpu().numpy()
    fp = fingerprint if fingerprint is not None else engine.fingerprint()
    if resume is not True and init is not None and st.init is None:
        # a format-1 (round-2) checkpoint records no initialisation, so "auto" cannot
        # prove it belongs to this fit (a checkpoint must never change the model)
        import warnings
        warnings.warn(f"{dirpath}: checkpoint without an initialisation record (format 1); "
                      "resume='auto' does not use it (pass resume=True to continue from it)")
        return 0, None, None
    why = mismatch(st, rank, reg, implicit, alpha, fp, ids,
                   init=None if resume is True else init)
    if why is None and st.iteration > max_iter:
        why = f"checkpoint is at iteration {st.iteration} > maxIter {max_iter}"
    if why is not None:
        if resume is True:
            raise ValueError(f"checkpoint in {dirpath} does not match this fit: {why}")
        return 0, None, None
    return st.iteration, st.U, (st.V if st.iteration == max_iter else None)


def resume_point_agreed(dirpath: Optional[str], resume, engine, rank: int, reg: float,
                        implicit: bool, alpha: float, max_iter: int, init: Optional[dict],
                        group, device):
    """resume_point for the ranks of a process group: every rank computes the
    fingerprint (a collective), process 0 alone reads the checkpoint and decides, and
    the decision — start iteration, error — and the factors are broadcast, so every
    rank starts at the same iteration from the same state (or every rank raises)."""
    import torch
    import torch.distributed as dist
    from .distributed import broadcast_capped
    if not resume or not dirpath:
        return 0, None, None
    fp = engine.fingerprint()  # collective: every rank
    proc = dist.get_rank(group)
    start, U, V, err = 0, None, None, None
    if proc == 0:
        # any failure (a mismatch, a missing or unreadable generation directory, a
        # malformed JSON) is broadcast, so every rank raises instead of waiting
        try:
            start, U, V = resume_point(dirpath, resume, engine, rank, reg, implicit, alpha,
                                       max_iter, init, fingerprint=fp)
        except Exception as e:  # noqa: BLE001 - re-raised on every rank below
            err = (type(e).__name__, str(e))
    head = [start, V is not None, err]
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast_object_list(head, src=src, group=group)
    start, has_v, err = head
    if err is not None:
        kind, msg = err
        raise (ValueError if kind == "ValueError" else RuntimeError)(
            msg if kind == "ValueError" else f"checkpoint in {dirpath} unreadable: {kind}: {msg}")
    if start == 0 and not has_v:
        return 0, None, None

    def bcast(F, n):
        t = (torch.as_tensor(F).to(device, torch.float32).contiguous() if proc == 0 else
             torch.empty((n, rank), dtype=torch.float32, device=device))
        return broadcast_capped(t, src, "checkpoint factors", group)

    U = bcast(U, engine.n_users)
    V = bcast(V, engine.n_items) if has_v else None
    return start, U, V


def maybe_save(dirpath: Optional[str], interval: int, it_done: int, engine, rank: int,
               reg: float, implicit: bool, alpha: float, writer: bool = True,
               init: Optional[dict] = None) -> None:
    """After iteration `it_done` (1-based count): write when it is a multiple of
    `interval` (Spark's checkpointInterval; <= 0 disables).  check_status() and
    fingerprint() run on every rank (collectives of a sharded engine); only the
    writer fetches the factors to the host (without caching dense copies)."""
    if not dirpath or interval is None or interval <= 0 or it_done % interval != 0:
        return
    engine.check_status()  # never checkpoint the state of a failed solve
    data = engine.fingerprint()
    if not writer:
        return
    uids, U = engine.user_factors(cache=False)
    iids, V = engine.item_factors(cache=False)
    save(dirpath, it_done, rank, reg, implicit, alpha, data, uids.cpu().numpy(),
         U.float().cpu().numpy(), iids.cpu().numpy(), V.float().cpu().numpy(), init=init)
