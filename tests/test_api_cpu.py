"""Host-side behaviour of the ml / mllib surfaces that needs no GPU: parameter
validation (Spark's ALSParams validators and error conditions), id checks
(ALS.checkIntegers), input adapters, and the MovieLens parsers/split."""
import gzip
import os

import numpy as np
import pandas as pd
import pytest

from als_mi355x import datasets
from als_mi355x._data import check_integers, columns_of
from als_mi355x.ml.recommendation import ALS as MLALS
from als_mi355x.mllib.recommendation import ALS as MLlibALS
from als_mi355x.mllib.recommendation import Rating, compute_error

HERE = os.path.dirname(os.path.abspath(__file__))
DF = pd.DataFrame({"user": [0, 1, 2], "item": [0, 1, 1], "rating": [1.0, 2.0, 3.0]})


@pytest.mark.parametrize("kw,exc", [
    (dict(rank=0), ValueError), (dict(maxIter=-1), ValueError), (dict(regParam=-0.1), ValueError),
    (dict(alpha=-1.0), ValueError), (dict(coldStartStrategy="zero"), ValueError),
    (dict(numUserBlocks=0), ValueError), (dict(nonnegative=True), NotImplementedError),
    (dict(rank=129), NotImplementedError)])
def test_ml_param_validation(kw, exc):
    with pytest.raises(exc):
        MLALS(**kw).fit(DF)


def test_ml_unknown_kwarg_and_accessors():
    with pytest.raises(TypeError):
        MLALS(rnak=3)
    als = MLALS().setRank(7).setMaxIter(3).setRegParam(0.5).setImplicitPrefs(True).setAlpha(2.0)
    assert (als.getRank(), als.getMaxIter(), als.getRegParam(), als.getImplicitPrefs(),
            als.getAlpha()) == (7, 3, 0.5, True, 2.0)
    assert als.getColdStartStrategy() == "nan" and als.getUserCol() == "user"
    als.setNumBlocks(4)
    assert als.getNumUserBlocks() == 4 and als.getNumItemBlocks() == 4


def test_ml_missing_column():
    with pytest.raises(ValueError, match="no column"):
        MLALS(userCol="uid").fit(DF)


@pytest.mark.parametrize("kw,exc", [(dict(rank=0), ValueError), (dict(iterations=-1), ValueError),
                                    (dict(lambda_=-1.0), ValueError),
                                    (dict(nonnegative=True), NotImplementedError)])
def test_mllib_param_validation(kw, exc):
    args = dict(rank=4)
    args.update(kw)
    with pytest.raises(exc):
        MLlibALS.train([(0, 0, 1.0)], **args)


def test_check_integers_spark_semantics():
    assert check_integers(np.array([1.0, 2.0]), "user").tolist() == [1, 2]
    with pytest.raises(ValueError, match="fractional"):
        check_integers(np.array([1.5]), "user")
    with pytest.raises(ValueError, match="Integer range"):
        check_integers(np.array([2 ** 31], dtype=np.int64), "item")
    with pytest.raises(ValueError):
        check_integers(np.array([np.nan]), "item")


def test_columns_of_adapters():
    trip = [(1, 2, 3.0), (4, 5, 6.0)]
    for ds in (trip, np.array(trip), [Rating(*t) for t in trip],
               {"user": [1, 4], "item": [2, 5], "rating": [3.0, 6.0]},
               pd.DataFrame(trip, columns=["user", "item", "rating"])):
        u, i, r = columns_of(ds, ("user", "item", "rating"))
        assert list(u) == [1, 4] and list(i) == [2, 5] and list(r) == [3.0, 6.0]


def test_host_compute_error_matches_kat():
    import json
    kat = json.load(open(os.path.join(HERE, "golden", "compute_error_kat.json")))
    for case in kat["cases"]:
        assert float("%.12g" % compute_error(case["predicted"], case["actual"])) == case["expected"]


def test_movielens_parsers(tmp_path):
    p = tmp_path / "ratings.dat.gz"
    with gzip.open(p, "wt") as f:
        f.write("1::1193::5::978300760\n1::914::3::978301968\n2::1::4.5::1\n")
    u, i, r = datasets.load_ratings(str(p))
    assert u.tolist() == [1, 1, 2] and i.tolist() == [1193, 914, 1] and r.tolist() == [5, 3, 4.5]
    c = tmp_path / "ratings.csv"
    c.write_text("userId,movieId,rating,timestamp\n1,31,2.5,1260759144\n1,1029,3.0,1\n")
    u, i, r = datasets.load_ratings(str(c))
    assert u.tolist() == [1, 1] and i.tolist() == [31, 1029] and r.tolist() == [2.5, 3.0]
    m = tmp_path / "movies.dat"
    m.write_text("1::Toy Story (1995)::Animation\n2::Jumanji (1995)::Adventure\n")
    assert datasets.load_movies(str(m)) == [(1, "Toy Story (1995)"), (2, "Jumanji (1995)")]
    assert datasets.get_ratings_tuple("1::1193::5::978300760") == (1, 1193, 5.0)


def test_random_split_proportions_and_determinism():
    a = datasets.random_split(100000, (6, 2, 2), seed=0)
    b = datasets.random_split(100000, (6, 2, 2), seed=0)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    sizes = [len(x) for x in a]
    assert sum(sizes) == 100000
    assert abs(sizes[0] / 1e5 - 0.6) < 0.01 and abs(sizes[1] / 1e5 - 0.2) < 0.01
    assert len(np.intersect1d(a[0], a[1])) == 0


def test_synthetic_generator_shape_cpu():
    u, i, r = datasets.synthetic(300, 200, 6000, seed=3, device="cpu")
    assert u.numel() == 6000
    keys = u.long() * 200 + i.long()
    assert keys.unique().numel() == 6000  # no duplicate pairs
    assert float(r.min()) >= 0.5 and float(r.max()) <= 5.0
    assert int(i.max()) < 200 and int(u.max()) < 300
    u2, i2, r2 = datasets.synthetic(300, 200, 6000, seed=3, device="cpu")
    assert (u == u2).all() and (i == i2).all() and (r == r2).all()


def test_blocked_generator_shards_reproduce_single_process():
    """configs[3]'s generator: exact nnz, no duplicate pairs, min user degree 20, and
    the union of the user-range shards equals the single-process dataset (strong
    scaling generates one global dataset)."""
    import numpy as np
    from als_mi355x import datasets as D
    kw = dict(n_users=6000, n_items=2000, nnz=300_000, seed=3, device="cpu",
              block_ratings=1 << 15)
    u, i, r = D.synthetic_blocked(**kw)
    assert u.numel() == 300_000
    keys = u.long() * 2000 + i.long()
    assert keys.unique().numel() == keys.numel()
    assert np.bincount(u.numpy()).min() >= 20
    assert float(r.min()) >= 0.5 and float(r.max()) <= 5.0
    parts = [D.synthetic_blocked(user_begin=6000 * w // 4, user_end=6000 * (w + 1) // 4, **kw)
             for w in range(4)]
    a = np.stack([u.numpy(), i.numpy(), r.numpy().view(np.int32)], 1)
    b = np.concatenate([np.stack([x.numpy(), y.numpy(), z.numpy().view(np.int32)], 1)
                        for x, y, z in parts])
    np.testing.assert_array_equal(a[np.lexsort((a[:, 1], a[:, 0]))],
                                  b[np.lexsort((b[:, 1], b[:, 0]))])
