"""Loaded files through a GPU fit: the reference's input path
(RecommenderSystem.py:16-39: `::` ratings/movies files parsed into tuples) and the
ml-latest-small CSV of BASELINE configs[0], written to disk from synthetic data of
the documented shapes (the real files are not in the container), read back by
`datasets.load_ratings` / `load_movies`, and fitted on the GPU against the C oracle
from the same seeded start."""
import gzip
import os

import numpy as np
import pytest

import als_mi355x.datasets as D
import als_mi355x.engine as E
from helpers import oracle_train_c, rel_row_err, report

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _seeded_u0(u, i, r, rank, seed):
    core = E.ALSCore(u, i, r, device=DEV)
    core.init_factors(rank, seed=seed)
    return core.U[:, :rank].cpu().numpy()


def test_ml_latest_small_csv_fit(tmp_path):
    """BASELINE configs[0]: ml-latest-small shape (610 x 9,724, 100,836 half-star
    ratings) as ratings.csv + movies.csv, ml ALS rank 10, maxIter 10, regParam 0.1."""
    import pandas as pd
    from als_mi355x.ml.recommendation import ALS
    n_u, n_i, nnz, half, seed = D.CONFIGS["ml_latest_small"]
    u, i, r = D.synthetic(n_u, n_i, nnz, seed=seed, half_stars=half, device=DEV)
    u, i, r = (u + 1).cpu().numpy(), (i + 1).cpu().numpy(), r.cpu().numpy()
    path = tmp_path / "ratings.csv"
    with open(path, "w") as f:
        f.write("userId,movieId,rating,timestamp\n")
        for a, b, c in zip(u.tolist(), i.tolist(), r.tolist()):
            f.write(f"{a},{b},{c:.1f},964982703\n")
    with open(tmp_path / "movies.csv", "w") as f:
        f.write("movieId,title,genres\n")
        for m in range(1, n_i + 1):
            f.write(f'{m},"Movie {m}, The (1995)",Drama|Comedy\n')
    lu, li, lr = D.load_ratings(str(path))
    movies = D.load_movies(str(tmp_path / "movies.csv"))
    assert len(lu) == nnz and len(movies) == n_i and movies[0] == (1, "Movie 1, The (1995)")
    np.testing.assert_array_equal(lr, r)
    model = ALS(rank=10, maxIter=10, regParam=0.1, seed=5).fit(
        pd.DataFrame({"user": lu, "item": li, "rating": lr}))
    U, V, umap, imap, uids, iids = oracle_train_c(lu, li, lr, 10, 10, 0.1,
                                                  _seeded_u0(lu, li, lr, 10, 5))
    ids, Uf = model.engine.user_factors()
    np.testing.assert_array_equal(ids.cpu().numpy(), uids)
    err = rel_row_err(Uf.cpu().numpy(), U)
    report("configs0_ml_latest_small_csv_fit_rel_err", err)
    assert err <= 1e-4


def test_movielens_dat_gz_fit(tmp_path):
    """The reference's `::` files (ratings.dat.gz with timestamps, movies.dat), lab-4
    shape, mllib ALS.train rank 8 as at RecommenderSystem.py:148."""
    from als_mi355x.mllib.recommendation import ALS
    n_u, n_i, nnz, half, seed = D.CONFIGS["ml1m_lab4"]
    u, i, r = D.synthetic(n_u, n_i, nnz, seed=seed, half_stars=half, device=DEV)
    u, i, r = (u + 1).cpu().numpy(), (i + 1).cpu().numpy(), r.cpu().numpy()
    with gzip.open(tmp_path / "ratings.dat.gz", "wt") as f:
        for a, b, c in zip(u.tolist(), i.tolist(), r.tolist()):
            f.write(f"{a}::{b}::{int(c)}::978300760\n")
    with open(tmp_path / "movies.dat", "w") as f:
        for m in range(1, n_i + 1):
            f.write(f"{m}::Movie {m} (2000)::Drama\n")
    lu, li, lr = D.load_ratings(str(tmp_path / "ratings.dat.gz"))
    movies = D.load_movies(str(tmp_path / "movies.dat"))
    assert len(lu) == nnz and movies[2] == (3, "Movie 3 (2000)")
    assert D.get_ratings_tuple("1::1193::5::978300760") == (1, 1193, 5.0)
    model = ALS.train(list(zip(lu.tolist(), li.tolist(), lr.tolist())), 8, seed=5,
                      iterations=5, lambda_=0.1)
    U, V, umap, imap, uids, iids = oracle_train_c(lu, li, lr, 8, 5, 0.1,
                                                  _seeded_u0(lu, li, lr, 8, 5))
    _, Uf = model.engine.user_factors()
    assert rel_row_err(Uf.cpu().numpy(), U) <= 1e-4
