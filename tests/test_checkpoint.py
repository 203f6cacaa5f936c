"""Factor checkpoints and resume (checkpoint.py).

CPU: the file format, atomic replacement and the matching rules, on a stand-in
engine.  GPU: an ALSCore fit interrupted at a checkpoint and resumed gives the
uninterrupted fit's factors bit for bit (the kernels are deterministic), and the
ml surface resumes through setCheckpointDir."""
import os

import numpy as np
import pytest
import torch

from als_mi355x import checkpoint as C

DEV = "cuda:0"


class _Eng:
    def __init__(self, ids, U, V, data):
        self.ids, self.U, self.V, self.data = ids, U, V, data

    def user_factor_ids(self):
        return torch.as_tensor(self.ids)

    def fingerprint(self):
        return dict(self.data)

    def user_factors(self, cache=True):
        return torch.as_tensor(self.ids), torch.as_tensor(self.U)

    def item_factors(self, cache=True):
        return torch.arange(self.V.shape[0], dtype=torch.int32), torch.as_tensor(self.V)

    def check_status(self):
        pass


def _eng(seed=0):
    rng = np.random.default_rng(seed)
    ids = np.array([-3, 0, 7, 12], np.int32)
    return _Eng(ids, rng.standard_normal((4, 3)).astype(np.float32),
                rng.standard_normal((5, 3)).astype(np.float32),
                {"nnz": 20, "n_users": 4, "n_items": 5, "rating_bits": 123, "item_id_sum": 10})


def test_save_interval_and_round_trip(tmp_path):
    e = _eng()
    d = str(tmp_path / "ck")
    C.maybe_save(d, 3, 2, e, 3, 0.1, False, 1.0)  # not a multiple of 3: nothing written
    assert C.load(d) is None
    C.maybe_save(d, 3, 3, e, 3, 0.1, False, 1.0)
    st = C.load(d)
    assert st.iteration == 3 and st.rank == 3 and st.data == e.data
    np.testing.assert_array_equal(st.U, e.U)
    np.testing.assert_array_equal(st.V, e.V)
    np.testing.assert_array_equal(st.user_ids, e.ids)
    assert not [f for f in os.listdir(d) if ".tmp" in f]
    C.maybe_save(d, -1, 4, e, 3, 0.1, False, 1.0)  # checkpointInterval -1: disabled
    assert C.load(d).iteration == 3
    C.maybe_save(d, 3, 6, _eng(1), 3, 0.1, False, 1.0)  # a new generation replaces the old
    assert C.load(d).iteration == 6
    assert len([f for f in os.listdir(d) if f.startswith("gen-")]) == 1


def test_save_killed_before_commit_keeps_previous_state(tmp_path, monkeypatch):
    """A save that dies after writing the new generation's files but before the JSON
    commit leaves the previous checkpoint whole: its iteration AND its factors."""
    d = str(tmp_path / "ck")
    old = _eng(0)
    C.maybe_save(d, 2, 2, old, 3, 0.1, False, 1.0, init={"seed": 1})
    real_replace = os.replace

    def dying_replace(src, dst):
        if dst.endswith(C.STATE):
            raise KeyboardInterrupt("killed before the commit")
        return real_replace(src, dst)

    monkeypatch.setattr(C.os, "replace", dying_replace)
    with pytest.raises(KeyboardInterrupt):
        C.maybe_save(d, 2, 4, _eng(5), 3, 0.1, False, 1.0, init={"seed": 1})
    monkeypatch.setattr(C.os, "replace", real_replace)
    st = C.load(d)
    assert st.iteration == 2
    np.testing.assert_array_equal(st.U, old.U)
    np.testing.assert_array_equal(st.V, old.V)
    # the next completed save commits and clears the orphaned generation
    C.maybe_save(d, 2, 4, _eng(5), 3, 0.1, False, 1.0, init={"seed": 1})
    assert C.load(d).iteration == 4
    assert len([f for f in os.listdir(d) if f.startswith("gen-")]) == 1
    assert not [f for f in os.listdir(d) if f.endswith(".tmp")]


def test_auto_resume_requires_the_same_initialisation(tmp_path):
    """Spark: a checkpoint dir never changes the model.  "auto" resumes only a fit with
    the same seed (or the same explicit U0); resume=True continues regardless."""
    e = _eng()
    d = str(tmp_path / "ck")
    C.maybe_save(d, 2, 2, e, 3, 0.1, False, 1.0, init=C.init_key(7, None))
    assert C.resume_point(d, "auto", e, 3, 0.1, False, 1.0, 10, C.init_key(7, None))[0] == 2
    assert C.resume_point(d, "auto", e, 3, 0.1, False, 1.0, 10, C.init_key(8, None)) == \
        (0, None, None)
    U0 = np.ones((4, 3), np.float32)
    assert C.resume_point(d, "auto", e, 3, 0.1, False, 1.0, 10, C.init_key(7, U0)) == \
        (0, None, None)
    assert C.resume_point(d, True, e, 3, 0.1, False, 1.0, 10, C.init_key(8, None))[0] == 2


def test_format1_checkpoint_auto_skips_with_warning_and_is_cleaned(tmp_path):
    """A round-2 (format-1) checkpoint has its files next to the JSON and no
    initialisation record: "auto" skips it with a warning, resume=True continues from
    it, and the first format-2 save removes the old top-level files."""
    import json
    e = _eng()
    d = tmp_path / "ck"
    d.mkdir()
    for name, arr in ((C.IDS, e.ids), (C.FACTORS, e.U), (C.IIDS, np.arange(5, dtype=np.int32)),
                      (C.IFACTORS, e.V)):
        np.save(d / name, arr, allow_pickle=False)
    (d / C.STATE).write_text(json.dumps({"format": 1, "iteration": 2, "rank": 3, "regParam": 0.1,
                                         "implicitPrefs": False, "alpha": 1.0, "data": e.data}))
    with pytest.warns(UserWarning, match="initialisation record"):
        assert C.resume_point(str(d), "auto", e, 3, 0.1, False, 1.0, 10,
                              C.init_key(1, None)) == (0, None, None)
    start, U, _ = C.resume_point(str(d), True, e, 3, 0.1, False, 1.0, 10, C.init_key(1, None))
    assert start == 2
    np.testing.assert_array_equal(U, e.U)
    C.maybe_save(str(d), 1, 3, e, 3, 0.1, False, 1.0, init=C.init_key(1, None))
    assert sorted(p.name for p in d.iterdir() if p.suffix == ".npy") == []
    assert C.load(str(d)).iteration == 3


def test_resume_point_rules(tmp_path):
    e = _eng()
    d = str(tmp_path / "ck")
    assert C.resume_point(d, "auto", e, 3, 0.1, False, 1.0, 10) == (0, None, None)
    with pytest.raises(ValueError, match="no ALS checkpoint"):
        C.resume_point(d, True, e, 3, 0.1, False, 1.0, 10)
    C.maybe_save(d, 2, 4, e, 3, 0.1, False, 1.0)
    start, U, V = C.resume_point(d, True, e, 3, 0.1, False, 1.0, 10)
    assert start == 4 and V is None
    np.testing.assert_array_equal(U, e.U)
    start, U, V = C.resume_point(d, True, e, 3, 0.1, False, 1.0, 4)  # at maxIter: V too
    assert start == 4
    np.testing.assert_array_equal(V, e.V)
    assert C.resume_point(d, False, e, 3, 0.1, False, 1.0, 10) == (0, None, None)
    bad = [(dict(rank=4), "rank"), (dict(reg=0.2), "regParam"), (dict(implicit=True), "regParam"),
           (dict(max_iter=3), "maxIter")]
    for kw, msg in bad:
        a = dict(rank=3, reg=0.1, implicit=False, alpha=1.0, max_iter=10)
        a.update(kw)
        with pytest.raises(ValueError, match=msg):
            C.resume_point(d, True, e, a["rank"], a["reg"], a["implicit"], a["alpha"],
                           a["max_iter"])
        assert C.resume_point(d, "auto", e, a["rank"], a["reg"], a["implicit"], a["alpha"],
                              a["max_iter"]) == (0, None, None)
    other = _eng()
    other.data["rating_bits"] = 124
    with pytest.raises(ValueError, match="ratings differ"):
        C.resume_point(d, True, other, 3, 0.1, False, 1.0, 10)
    other = _eng()
    other.ids = np.array([-3, 0, 7, 13], np.int32)
    with pytest.raises(ValueError, match="user ids differ"):
        C.resume_point(d, True, other, 3, 0.1, False, 1.0, 10)


@pytest.mark.gpu
@pytest.mark.parametrize("implicit", [False, True])
def test_gpu_resume_bit_exact(tmp_path, implicit):
    from als_mi355x.engine import ALSCore
    from helpers import planted
    u, i, r = planted(400, 250, density=0.05, seed=17, heavy_items=(2,), dup=5)
    u = (u - 100).astype(np.int32)
    full = ALSCore(u, i, r, device=DEV).fit(12, 6, 0.1, implicit, 4.0, seed=3)
    d = str(tmp_path / "ck")
    ALSCore(u, i, r, device=DEV).fit(12, 4, 0.1, implicit, 4.0, seed=3, checkpoint_dir=d,
                                     checkpoint_interval=2)
    assert C.load(d).iteration == 4
    res = ALSCore(u, i, r, device=DEV).fit(12, 6, 0.1, implicit, 4.0, seed=999, checkpoint_dir=d,
                                           checkpoint_interval=0, resume=True)
    assert torch.equal(res.U, full.U) and torch.equal(res.V, full.V)
    # other ratings: strict resume refuses, "auto" starts fresh
    r2 = r.copy()
    r2[0] += 1.0
    with pytest.raises(ValueError, match="ratings differ"):
        ALSCore(u, i, r2, device=DEV).fit(12, 6, 0.1, implicit, 4.0, checkpoint_dir=d,
                                          resume=True)
    fresh = ALSCore(u, i, r2, device=DEV).fit(12, 6, 0.1, implicit, 4.0, seed=3,
                                              checkpoint_dir=d, checkpoint_interval=0,
                                              resume="auto")
    ref = ALSCore(u, i, r2, device=DEV).fit(12, 6, 0.1, implicit, 4.0, seed=3)
    assert torch.equal(fresh.U, ref.U)


@pytest.mark.gpu
def test_gpu_ml_fit_resumes_from_checkpoint_dir(tmp_path):
    import pandas as pd
    from als_mi355x.ml.recommendation import ALS
    from helpers import planted
    u, i, r = planted(300, 200, density=0.05, seed=19)
    df = pd.DataFrame({"user": u, "item": i, "rating": r})
    ref = ALS(rank=8, maxIter=6, regParam=0.1, seed=1).fit(df)
    d = str(tmp_path / "ck")
    ALS(rank=8, maxIter=3, regParam=0.1, seed=1, checkpointInterval=3).setCheckpointDir(d).fit(df)
    assert C.load(d).iteration == 3
    m = ALS(rank=8, maxIter=6, regParam=0.1, seed=1, checkpointInterval=3).setCheckpointDir(d).fit(df)
    assert torch.equal(m.engine.U, ref.engine.U) and torch.equal(m.engine.V, ref.engine.V)
    assert C.load(d).iteration == 6


def test_save_keeps_user_files_that_share_the_format1_names(tmp_path):
    """Same-named .npy files the user keeps in the checkpoint directory are not ours
    unless a format-1 checkpoint is being replaced: a save into a fresh directory (and
    over a format-2 checkpoint) leaves them alone."""
    e = _eng()
    d = tmp_path / "ck"
    d.mkdir()
    mine = np.arange(7, dtype=np.int32)
    np.save(d / C.FACTORS, mine, allow_pickle=False)
    C.maybe_save(str(d), 1, 1, e, 3, 0.1, False, 1.0, init=C.init_key(1, None))
    C.maybe_save(str(d), 1, 2, e, 3, 0.1, False, 1.0, init=C.init_key(1, None))
    np.testing.assert_array_equal(np.load(d / C.FACTORS), mine)
    assert C.load(str(d)).iteration == 2
