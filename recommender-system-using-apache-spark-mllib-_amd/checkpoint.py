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
    als_state.json      {"format": 1, "iteration": t, "rank", "regParam",
                         "implicitPrefs", "alpha", "data": fingerprint}
    user_ids.npy        int32 [n_users]   dense order (ascending ids)
    user_factors.npy    float32 [n_users, rank]
    item_ids.npy, item_factors.npy        the same for V (needed only when the
                        checkpoint is already at the requested iteration count:
                        V_t came from U_{t-1}, which is not kept)
Files are written to temporaries and renamed, the JSON last, so a job killed
mid-write leaves the previous checkpoint intact.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

STATE = "als_state.json"
IDS = "user_ids.npy"
FACTORS = "user_factors.npy"
IIDS = "item_ids.npy"
IFACTORS = "item_factors.npy"
FORMAT = 1


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


def _replace_npy(path: str, arr: np.ndarray) -> None:
    tmp = path + ".tmp.npy"
    np.save(tmp, arr, allow_pickle=False)
    os.replace(tmp, path)


def save(dirpath: str, iteration: int, rank: int, reg: float, implicit: bool, alpha: float,
         data: dict, user_ids, U, item_ids, V) -> None:
    """Write the state after `iteration` completed iterations."""
    os.makedirs(dirpath, exist_ok=True)
    for ids_name, f_name, ids, F in ((IDS, FACTORS, user_ids, U), (IIDS, IFACTORS, item_ids, V)):
        ids = np.ascontiguousarray(np.asarray(ids), dtype=np.int32)
        F = np.ascontiguousarray(np.asarray(F), dtype=np.float32)
        if F.shape != (ids.shape[0], rank):
            raise ValueError(f"factor table {F.shape} does not match {ids.shape[0]} ids x rank "
                             f"{rank}")
        _replace_npy(os.path.join(dirpath, ids_name), ids)
        _replace_npy(os.path.join(dirpath, f_name), F)
    meta = {"format": FORMAT, "iteration": int(iteration), "rank": int(rank),
            "regParam": float(reg), "implicitPrefs": bool(implicit), "alpha": float(alpha),
            "data": data}
    tmp = os.path.join(dirpath, STATE + ".tmp")
    with open(tmp, "w") as f:
        json.dump(meta, f)
    os.replace(tmp, os.path.join(dirpath, STATE))


def load(dirpath: str) -> Optional[State]:
    """The checkpoint in `dirpath`, or None when there is none."""
    p = os.path.join(dirpath, STATE)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        m = json.load(f)
    if m.get("format") != FORMAT:
        raise ValueError(f"{p}: unknown checkpoint format {m.get('format')}")
    arr = [np.load(os.path.join(dirpath, n), allow_pickle=False)
           for n in (IDS, FACTORS, IIDS, IFACTORS)]
    return State(int(m["iteration"]), int(m["rank"]), float(m["regParam"]),
                 bool(m["implicitPrefs"]), float(m["alpha"]), m["data"], *arr)


def mismatch(st: State, rank: int, reg: float, implicit: bool, alpha: float, data: dict,
             user_ids) -> Optional[str]:
    """Why `st` cannot seed this fit (None when it can)."""
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
    return None


def resume_point(dirpath: Optional[str], resume, engine, rank: int, reg: float, implicit: bool,
                 alpha: float, max_iter: int):
    """(start iteration, U0, V0) for engine.fit; U0/V0 None for a fresh start, V0 set
    only when the checkpoint is already at max_iter.  resume: False = start fresh;
    True = the checkpoint must exist and match (ValueError otherwise); "auto" = use
    it when it matches, else start fresh."""
    if not resume or not dirpath:
        return 0, None, None
    st = load(dirpath)
    if st is None:
        if resume is True:
            raise ValueError(f"no ALS checkpoint in {dirpath}")
        return 0, None, None
    ids = engine.user_factor_ids().cpu().numpy()
    why = mismatch(st, rank, reg, implicit, alpha, engine.fingerprint(), ids)
    if why is None and st.iteration > max_iter:
        why = f"checkpoint is at iteration {st.iteration} > maxIter {max_iter}"
    if why is not None:
        if resume is True:
            raise ValueError(f"checkpoint in {dirpath} does not match this fit: {why}")
        return 0, None, None
    return st.iteration, st.U, (st.V if st.iteration == max_iter else None)


def maybe_save(dirpath: Optional[str], interval: int, it_done: int, engine, rank: int,
               reg: float, implicit: bool, alpha: float, writer: bool = True) -> None:
    """After iteration `it_done` (1-based count): write when it is a multiple of
    `interval` (Spark's checkpointInterval; <= 0 disables)."""
    if not dirpath or interval is None or interval <= 0 or it_done % interval != 0:
        return
    engine.check_status()  # never checkpoint the state of a failed solve
    uids, U = engine.user_factors()
    iids, V = engine.item_factors()
    data = engine.fingerprint()
    if writer:
        save(dirpath, it_done, rank, reg, implicit, alpha, data, uids.cpu().numpy(),
             U.float().cpu().numpy(), iids.cpu().numpy(), V.float().cpu().numpy())
