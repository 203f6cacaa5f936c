"""The north-star surface on the GPU, against the oracle on small planted sets.

pyspark.ml.recommendation: ALS(...).fit(df) -> ALSModel with transform
(coldStartStrategy "nan" / "drop"), recommendForAllUsers / ForAllItems /
ForUserSubset / ForItemSubset, userFactors / itemFactors; and the mllib
facade's trainImplicit.  Every fit is reproduced by the fp64 oracle from the
SAME initial factors (the engine's seeded draw), factors within 1e-4 relative
per row (north_star), predictions within fp32 rounding, top-k ids identical
except where the oracle's scores tie within the 1e-4 factor bar.  Spark semantics restated in SURVEY.md App. A.
"""
import numpy as np
import pandas as pd
import pytest
import torch

import als_mi355x.engine as E
from als_mi355x.ml.recommendation import ALS
from als_mi355x.mllib import recommendation as mllib
from helpers import planted, rel_row_err
from oracle import als_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _seeded_u0(u, i, r, rank, seed):
    """The initial user factors ALSCore.fit draws for `seed` (unit-norm Gaussian rows)."""
    core = E.ALSCore(u, i, r, device=DEV)
    core.init_factors(rank, seed=seed)
    return core.U[:, :rank].cpu().numpy()


@pytest.fixture(scope="module")
def data():
    u, i, r = planted(300, 200, density=0.06, seed=3, id_gap=3)
    u = (u - 150).astype(np.int32)   # negative user ids are legal Spark Int ids
    return u, i, r


@pytest.fixture(scope="module")
def fitted(data):
    u, i, r = data
    df = pd.DataFrame({"user": u, "item": i, "rating": r})
    model = ALS(rank=8, maxIter=5, regParam=0.1, seed=42).fit(df)
    U0 = _seeded_u0(u, i, r, 8, 42)
    U, V, umap, imap, uids, iids = O.train(u + 150, i, r, 8, 5, 0.1, U0=U0)
    return model, (U, V, umap, imap, uids - 150, iids)


def test_ml_fit_factors_match_oracle(fitted):
    model, (U, V, _, _, uids, iids) = fitted
    uf, itf = model.userFactors, model.itemFactors
    assert list(uf.columns) == ["id", "features"]
    np.testing.assert_array_equal(uf["id"].to_numpy(), uids)
    np.testing.assert_array_equal(itf["id"].to_numpy(), iids)
    assert rel_row_err(np.stack(uf["features"].to_numpy()), U) <= 1e-4
    assert rel_row_err(np.stack(itf["features"].to_numpy()), V) <= 1e-4
    assert model.rank == 8


@pytest.mark.parametrize("strategy", ["nan", "drop"])
def test_ml_transform_cold_start(fitted, data, strategy):
    model, (U, V, umap, imap, uids, iids) = fitted
    u, i, _ = data
    rng = np.random.default_rng(5)
    qu = np.concatenate([rng.choice(u, 50), [10 ** 6, -(10 ** 6), int(u[0])]]).astype(np.int32)
    qi = np.concatenate([rng.choice(i, 50), [int(i[0]), int(i[1]), 10 ** 6]]).astype(np.int32)
    df = pd.DataFrame({"user": qu, "item": qi, "extra": np.arange(len(qu))})
    out = model.setColdStartStrategy(strategy).transform(df)
    ref = O.predict(U, V, umap, imap, qu + 150, qi)  # oracle maps are keyed by id + 150
    cold = np.isnan(ref)
    assert cold.sum() == 3
    if strategy == "nan":
        assert len(out) == len(df) and list(out.columns) == ["user", "item", "extra", "prediction"]
        got = out["prediction"].to_numpy()
        np.testing.assert_array_equal(np.isnan(got), cold)
    else:
        assert len(out) == len(df) - 3
        np.testing.assert_array_equal(out["extra"].to_numpy(), np.nonzero(~cold)[0])
        got = np.full(len(df), np.nan)
        got[out["extra"].to_numpy()] = out["prediction"].to_numpy()
    assert out["prediction"].dtype == np.float32
    np.testing.assert_allclose(got[~cold], ref[~cold], rtol=1e-4, atol=1e-5)
    model.setColdStartStrategy("nan")


def _check_recs(df, key_col, keys_ref, Q, Vm, other_ids, k):
    assert list(df.columns) == [key_col, "recommendations"]
    np.testing.assert_array_equal(df[key_col].to_numpy(), keys_ref)
    ref_i, ref_s = O.topk(Q, Vm, k)
    S = Q.astype(np.float64) @ Vm.astype(np.float64).T
    for row, recs in enumerate(df["recommendations"]):
        assert len(recs) == min(k, Vm.shape[0])
        got_ids = np.array([a for a, _ in recs])
        got_sc = np.array([b for _, b in recs])
        assert np.all(np.diff(got_sc) <= 1e-6)  # rating descending
        ref_ids = other_ids[ref_i[row, :len(recs)]]
        for p in np.nonzero(got_ids != ref_ids)[0]:  # only fp ties may swap
            j = int(np.searchsorted(other_ids, got_ids[p]))
            assert abs(S[row, j] - ref_s[row, p]) <= 1e-4 * max(1.0, abs(ref_s[row, p]))
        np.testing.assert_allclose(got_sc, ref_s[row, :len(recs)], rtol=1e-4, atol=1e-4)


def test_ml_recommend_for_all_users_and_items(fitted):
    model, (U, V, _, _, uids, iids) = fitted
    _check_recs(model.recommendForAllUsers(10), "user", uids, U, V, iids, 10)
    _check_recs(model.recommendForAllItems(7), "item", iids, V, U, uids, 7)
    # more recommendations than items: every item once
    big = model.recommendForAllUsers(len(iids) + 5)
    assert all(len(x) == len(iids) for x in big["recommendations"])


def test_ml_recommend_for_subsets(fitted, data):
    model, (U, V, _, _, uids, iids) = fitted
    sub = pd.DataFrame({"user": [int(uids[3]), int(uids[3]), 10 ** 7, int(uids[0])]})
    df = model.recommendForUserSubset(sub, 5)
    rows = np.array([0, 3])
    _check_recs(df, "user", uids[rows], U[rows], V, iids, 5)
    subi = pd.DataFrame({"item": [int(iids[-1]), -5]})
    dfi = model.recommendForItemSubset(subi, 4)
    _check_recs(dfi, "item", iids[-1:], V[-1:], U, uids, 4)
    empty = model.recommendForUserSubset(pd.DataFrame({"user": [10 ** 7]}), 5)
    assert len(empty) == 0


def test_mllib_train_implicit_matches_oracle():
    u, i, r = planted(250, 180, density=0.07, seed=8)
    r = (r - 2.5).astype(np.float32)  # implicit data: negative preferences too
    trip = list(zip(u.tolist(), i.tolist(), r.tolist()))
    model = mllib.ALS.trainImplicit(trip, 12, iterations=4, lambda_=0.05, alpha=8.0, seed=9)
    U0 = _seeded_u0(u, i, r, 12, 9)
    U, V, umap, imap, uids, iids = O.train(u, i, r, 12, 4, 0.05, implicit=True, alpha=8.0, U0=U0)
    feats = model.userFeatures()
    assert [a for a, _ in feats] == list(uids)
    assert rel_row_err(np.array([f for _, f in feats]), U) <= 1e-4
    pf = model.productFeatures()
    assert rel_row_err(np.array([f for _, f in pf]), V) <= 1e-4
    # mllib predictAll: inner join, fp64 dot of the fp32 factors
    pairs = [(int(u[0]), int(i[0])), (10 ** 6, int(i[0])), (int(u[1]), int(i[1]))]
    preds = model.predictAll(pairs)
    assert [(p.user, p.product) for p in preds] == [pairs[0], pairs[2]]
    ref = O.predict(U, V, umap, imap, [pairs[0][0], pairs[2][0]], [pairs[0][1], pairs[2][1]])
    np.testing.assert_allclose([p.rating for p in preds], ref, rtol=1e-4, atol=1e-6)
    recs = model.recommendProducts(int(u[0]), 5)
    assert [x.user for x in recs] == [int(u[0])] * 5
    with pytest.raises(KeyError):
        model.recommendProducts(10 ** 6, 5)


def test_mllib_train_rmse_and_compute_error_agree():
    """R:103-129 computeError over predictAll output == the fused device RMSE (K4)."""
    u, i, r = planted(200, 150, density=0.08, seed=12)
    trip = list(zip(u.tolist(), i.tolist(), r.tolist()))
    model = mllib.ALS.train(trip, 6, seed=5, iterations=3, lambda_=0.1)
    held = trip[::7] + [(10 ** 6, 1, 3.0)]  # one cold pair: dropped by the join
    err = mllib.compute_error(model.predictAll([(a, b) for a, b, _ in held]), held)
    assert abs(model.rmse(held) - err) <= 1e-9
    assert abs(err - O.compute_error(model.predictAll([(a, b) for a, b, _ in held]), held)) == 0.0


def test_ml_params_errors():
    with pytest.raises(ValueError):
        ALS(rank=0).fit(pd.DataFrame({"user": [1], "item": [1], "rating": [1.0]}))
    with pytest.raises(ValueError):
        ALS(coldStartStrategy="zero").fit(pd.DataFrame({"user": [1], "item": [1], "rating": [1.0]}))
    with pytest.raises(ValueError):
        ALS().fit(pd.DataFrame({"user": [1.5], "item": [1], "rating": [1.0]}))


def test_engine_ids_beyond_compact_range():
    """Ids far from 0 (and negative) use an offset map; predictions unchanged."""
    u, i, r = planted(120, 90, density=0.1, seed=4)
    base = E.ALSCore(u, i, r, device=DEV).fit(6, 2, 0.1, seed=1)
    shifted = E.ALSCore(u.astype(np.int64) + 2_000_000_000 - 200, i - 50, r, device=DEV)
    shifted.fit(6, 2, 0.1, seed=1)
    assert shifted.uidx.offset != 0 and shifted.iidx.offset != 0
    p0 = base.predict(u[:100], i[:100]).cpu().numpy()
    p1 = shifted.predict(u[:100].astype(np.int64) + 2_000_000_000 - 200, i[:100] - 50)
    np.testing.assert_array_equal(p0, p1.cpu().numpy())
    ids, _ = shifted.user_factors()
    assert int(ids.min()) == int(u.min()) + 2_000_000_000 - 200
    assert torch.isnan(shifted.predict([0], [0])).all()


def test_topk_non_finite_factors_leave_no_bogus_ids():
    """Scores involving a NaN factor row are NaN; the kernel never ranks them, so a query
    row with NaN factors gets no recommendations (empty slots, score -inf) and a NaN item
    is never recommended.  The ml / mllib surfaces drop the empty slots instead of
    turning their placeholder index into an id."""
    rng = np.random.default_rng(4)
    U = rng.normal(size=(40, 12)).astype(np.float32)
    V = rng.normal(size=(30, 12)).astype(np.float32)
    U[5] = np.nan
    V[7] = np.nan
    uids = np.arange(40, dtype=np.int32) * 2 - 11   # negative ids included
    iids = np.arange(30, dtype=np.int32) * 3 + 1
    core = E.ALSCore.from_factors(uids, U, iids, V, device=DEV)
    keys, ids, sc = core.recommend_all(10, True)
    sc = sc.cpu().numpy()
    ids = ids.cpu().numpy()
    assert np.all(np.isneginf(sc[5]))
    ok = np.isfinite(sc)
    assert ok[np.arange(40) != 5].all()
    assert not np.any(ids[ok] == iids[7])
    S = U.astype(np.float64) @ V.astype(np.float64).T
    S[:, 7] = -np.inf
    for t in range(40):
        if t == 5:
            continue
        ref = np.lexsort((np.arange(30), -S[t]))[:10]
        np.testing.assert_array_equal(ids[t], iids[ref])
    model = mllib.MatrixFactorizationModel(core)
    assert model.recommendProducts(int(uids[5]), 10) == []
    recs = dict(model.recommendProductsForUsers(10))
    assert recs[int(uids[5])] == [] and len(recs[int(uids[0])]) == 10
    from als_mi355x.ml.recommendation import ALSModel
    lists = ALSModel._recs_df("user", *core.recommend_all(10, True))
    assert lists.loc[lists["user"] == uids[5], "recommendations"].iloc[0] == []
