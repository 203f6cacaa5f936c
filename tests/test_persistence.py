"""Model persistence in Spark's layout: round trips on the host.

Parity is against the restated upstream format (MatrixFactorizationModel.SaveLoadV1_0,
ALSModelWriter); no Spark-written model exists in the reference to pin it, so the
on-disk layout is "parity unpinned" beyond these self-consistency checks.
"""
import json
import os

import numpy as np
import pytest

from als_mi355x import persistence as P


def _factors(rng, n, k, lo=0, hi=10_000):
    ids = rng.choice(np.arange(lo, hi), size=n, replace=False).astype(np.int32)
    return ids, rng.standard_normal((n, k)).astype(np.float32)


def test_mllib_round_trip_bit_exact(tmp_path):
    rng = np.random.default_rng(0)
    uids, U = _factors(rng, 300, 8)
    pids, V = _factors(rng, 120, 8)
    path = str(tmp_path / "model")
    P.save_mllib(path, 8, uids, U, pids, V)
    meta = json.loads(open(os.path.join(path, "metadata", "part-00000")).readline())
    assert meta == {"class": P.MLLIB_CLASS, "version": "1.0", "rank": 8}
    rank, u2, U2, p2, V2 = P.load_mllib(path)
    assert rank == 8 and U2.dtype == np.float64
    ou, op = np.argsort(uids), np.argsort(pids)  # loaded in ascending id order
    np.testing.assert_array_equal(u2, uids[ou])
    np.testing.assert_array_equal(p2, pids[op])
    np.testing.assert_array_equal(U2.astype(np.float32), U[ou])  # fp32 -> fp64 -> fp32 exact
    np.testing.assert_array_equal(V2.astype(np.float32), V[op])


def test_ml_round_trip_and_params(tmp_path):
    rng = np.random.default_rng(1)
    uids, U = _factors(rng, 50, 5)
    iids, V = _factors(rng, 40, 5)
    path = str(tmp_path / "alsmodel")
    params = {"rank": 5, "regParam": 0.1, "coldStartStrategy": "drop"}
    P.save_ml(path, "ALS_0001", params, 5, uids, U, iids, V)
    meta = json.loads(open(os.path.join(path, "metadata", "part-00000")).readline())
    # DefaultParamsWriter: a parseable sparkVersion, the model's set params only, and
    # the model's defaults in defaultParamMap
    major, minor = (int(x) for x in meta["sparkVersion"].split(".")[:2])
    assert (major, minor) >= (2, 4)
    assert meta["defaultParamMap"] == P.ML_MODEL_DEFAULTS
    uid, p2, rank, u2, U2, i2, V2 = P.load_ml(path)
    assert uid == "ALS_0001" and p2 == {"coldStartStrategy": "drop"} and rank == 5
    assert U2.dtype == np.float32
    np.testing.assert_array_equal(U2, U[np.argsort(uids)])
    np.testing.assert_array_equal(V2, V[np.argsort(iids)])


def test_existing_path_and_overwrite(tmp_path):
    rng = np.random.default_rng(2)
    uids, U = _factors(rng, 4, 2)
    path = str(tmp_path / "m")
    P.save_mllib(path, 2, uids, U, uids, U)
    with pytest.raises(FileExistsError):
        P.save_mllib(path, 2, uids, U, uids, U)
    # a stale part file from an earlier (e.g. multi-partition) save must not survive
    stale = os.path.join(path, "data", "user", "part-00001.parquet")
    os.replace(os.path.join(path, "data", "user", "part-00000.parquet"), stale)
    P.save_mllib(path, 2, uids, 2 * U, uids, U, overwrite=True)
    assert not os.path.exists(stale)
    np.testing.assert_array_equal(P.load_mllib(path)[2].astype(np.float32),
                                  (2 * U)[np.argsort(uids)])
    open(str(tmp_path / "f"), "w").close()  # a plain file in the way
    with pytest.raises(FileExistsError):
        P.save_mllib(str(tmp_path / "f"), 2, uids, U, uids, U)


def test_wrong_class_and_bad_rank(tmp_path):
    rng = np.random.default_rng(3)
    uids, U = _factors(rng, 4, 3)
    path = str(tmp_path / "m")
    P.save_ml(path, "u", {}, 3, uids, U, uids, U)
    with pytest.raises(ValueError, match="not a"):
        P.load_mllib(path)
    meta = os.path.join(path, "metadata", "part-00000")
    d = json.loads(open(meta).readline())
    d["rank"] = 4
    open(meta, "w").write(json.dumps(d) + "\n")
    with pytest.raises(ValueError, match="expected rank 4"):
        P.load_ml(path)


def test_empty_side(tmp_path):
    path = str(tmp_path / "m")
    P.save_mllib(path, 3, np.zeros(0, np.int32), np.zeros((0, 3)), np.array([7], np.int32),
                 np.ones((1, 3)))
    rank, u2, U2, p2, V2 = P.load_mllib(path)
    assert u2.shape == (0,) and U2.shape == (0, 3) and p2.tolist() == [7]


@pytest.mark.gpu
def test_gpu_save_load_predict_and_topk_identical(tmp_path):
    """A model saved and loaded back predicts and recommends exactly as before (HIP path)."""
    from als_mi355x.ml.recommendation import ALSModel
    from als_mi355x.mllib.recommendation import ALS, MatrixFactorizationModel
    rng = np.random.default_rng(4)
    n_u, n_i = 200, 90
    mask = rng.random((n_u, n_i)) < 0.1
    mask[np.arange(n_u), rng.integers(0, n_i, n_u)] = True
    mask[rng.integers(0, n_u, n_i), np.arange(n_i)] = True
    u, i = np.nonzero(mask)
    r = rng.integers(1, 6, len(u)).astype(np.float32)
    model = ALS.train(np.stack([u * 3, i * 2 + 1, r], 1), 8, iterations=3, lambda_=0.1, seed=1)
    path = str(tmp_path / "mf")
    model.save(None, path)
    m2 = MatrixFactorizationModel.load(None, path)
    pu, pi = u[:500] * 3, i[:500] * 2 + 1
    np.testing.assert_array_equal(model.predictAllArrays(pu, pi), m2.predictAllArrays(pu, pi))
    a = model.recommendProductsForUsers(5)
    b = m2.recommendProductsForUsers(5)
    assert a == b
    assert np.isnan(m2.predictAllArrays([1], [0])[0])  # unknown ids stay unknown
    # ml layout: a model built over the same core round-trips too
    mlm = ALSModel(model.engine, {"rank": 8, "userCol": "user", "itemCol": "item",
                                  "predictionCol": "prediction", "coldStartStrategy": "nan"})
    mlm.save(str(tmp_path / "ml"))
    m3 = ALSModel.load(str(tmp_path / "ml"))
    np.testing.assert_array_equal(m3.engine.predict(pu, pi).cpu().numpy(),
                                  model.predictAllArrays(pu, pi))
