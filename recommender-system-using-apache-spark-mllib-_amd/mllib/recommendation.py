"""pyspark.mllib.recommendation-compatible facade: ALS.train / trainImplicit,
MatrixFactorizationModel, Rating.

This is the surface the reference script actually calls
(``from pyspark.mllib.recommendation import ALS`` at RecommenderSystem.py:132;
``ALS.train(trainingRDD, rank, seed=seed, iterations=iterations,
lambda_=regularizationParameter)`` at :148-149, :163, :218;
``model.predictAll(pairsRDD)`` at :150, :165, :222, :232).  Each call maps 1:1:
RDDs become Python iterables / numpy arrays / pandas frames / torch tensors,
and the arithmetic runs on the MI355X engine.

Semantics kept from upstream pyspark/mllib (``mllib/recommendation.py``,
``MatrixFactorizationModel.scala``):
  * ratings are (user, product, rating) triples; ratings cast to float32;
  * ``predictAll`` is an inner join: pairs with an unknown user or product are
    dropped; predictions are fp64 dots of the fp32 factors (``ddot``);
  * ``lambda_`` default 0.01, ``iterations`` default 5, ``blocks`` ignored
    (single CSR per side), ``nonnegative=True`` is out of scope.
"""
from __future__ import annotations

import zlib
from collections import namedtuple
from typing import Iterable, List, Optional

import numpy as np

from .. import engine as _engine
from .._data import check_integers, columns_of, to_float32

__all__ = ["ALS", "MatrixFactorizationModel", "Rating"]

_DEFAULT_SEED = zlib.crc32(b"org.apache.spark.mllib.recommendation.ALS")


class Rating(namedtuple("Rating", ["user", "product", "rating"])):
    """Represents a (user, product, rating) tuple (pyspark.mllib.recommendation.Rating)."""

    def __reduce__(self):
        return Rating, (int(self.user), int(self.product), float(self.rating))


def _triples(ratings):
    if hasattr(ratings, "columns") and {"user", "product", "rating"} <= set(ratings.columns):
        cols = ("user", "product", "rating")
        u, i, r = columns_of(ratings, cols)
    elif hasattr(ratings, "columns"):  # any 3-column frame, positional
        u, i, r = columns_of(ratings.to_numpy(), ("user", "product", "rating"))
    else:
        u, i, r = columns_of(ratings, ("user", "product", "rating"))
    return check_integers(u, "user"), check_integers(i, "product"), to_float32(r)


def _pairs(user_product):
    if hasattr(user_product, "to_numpy"):
        user_product = user_product.to_numpy()
    u, i = columns_of(user_product, ("user", "product"))
    return check_integers(u, "user"), check_integers(i, "product")


class MatrixFactorizationModel:
    """A matrix factorisation model trained by ALS; factors stay in HBM."""

    def __init__(self, core: "_engine.ALSCore"):
        self._core = core

    @property
    def rank(self) -> int:
        return self._core.rank

    @property
    def engine(self) -> "_engine.ALSCore":
        return self._core

    def predict(self, user: int, product: int) -> float:
        p = self._core.predict(np.array([user], np.int32), np.array([product], np.int32))
        v = float(p.cpu().numpy()[0])
        if np.isnan(v):
            raise KeyError(f"unknown user {user} or product {product}")
        return v

    def predictAll(self, user_product) -> List[Rating]:
        """Predicted Ratings for the (user, product) pairs whose ids are both known
        (inner join, as MatrixFactorizationModel.predict(RDD) does)."""
        u, i = _pairs(user_product)
        if len(u) == 0:
            return []
        p = self._core.predict(u, i).cpu().numpy()
        ok = ~np.isnan(p)
        return [Rating(int(a), int(b), float(c)) for a, b, c in zip(u[ok], i[ok], p[ok])]

    def predictAllArrays(self, users, products) -> np.ndarray:
        """fp64 predictions for arrays of ids (NaN where an id is unknown)."""
        return self._core.predict(check_integers(users, "user"),
                                  check_integers(products, "product")).cpu().numpy()

    def rmse(self, ratings) -> float:
        """computeError(predictAll(pairs), ratings) fused on the device (K4)."""
        u, i, r = _triples(ratings)
        rm, _ = self._core.rmse(u, i, r)
        return rm

    def userFeatures(self):
        ids, F = self._core.user_factors()
        F = F.double().cpu().numpy()
        return [(int(a), tuple(row)) for a, row in zip(ids.cpu().numpy(), F)]

    def productFeatures(self):
        ids, F = self._core.item_factors()
        F = F.double().cpu().numpy()
        return [(int(a), tuple(row)) for a, row in zip(ids.cpu().numpy(), F)]

    def _one(self, key, num, user_side):
        keys, ids, sc = self._core.recommend_subset([int(key)], int(num), user_side)
        if keys.numel() == 0:
            raise KeyError(f"unknown id {key}")
        ids, sc = ids.cpu().numpy()[0], sc.cpu().numpy()[0]
        return [Rating(key, int(a), float(s)) if user_side else Rating(int(a), key, float(s))
                for a, s in zip(ids, sc) if np.isfinite(s)]

    def recommendProducts(self, user: int, num: int) -> List[Rating]:
        return self._one(int(user), num, True)

    def recommendUsers(self, product: int, num: int) -> List[Rating]:
        return self._one(int(product), num, False)

    def recommendProductsForUsers(self, num: int):
        keys, ids, sc = self._core.recommend_all(int(num), True)
        keys, ids, sc = keys.cpu().numpy(), ids.cpu().numpy(), sc.cpu().numpy()
        return [(int(k), [Rating(int(k), int(a), float(s)) for a, s in zip(ri, rs)
                          if np.isfinite(s)])
                for k, ri, rs in zip(keys, ids, sc)]

    def save(self, sc, path: str, overwrite: bool = False) -> None:
        """MatrixFactorizationModel.save(sc, path) in Spark's layout (``sc`` is ignored)."""
        from .. import persistence
        uids, U = self._core.user_factors()
        pids, V = self._core.item_factors()
        persistence.save_mllib(path, self.rank, uids.cpu().numpy(), U.cpu().numpy(),
                               pids.cpu().numpy(), V.cpu().numpy(), overwrite=overwrite)

    @classmethod
    def load(cls, sc, path: str) -> "MatrixFactorizationModel":
        """MatrixFactorizationModel.load(sc, path): factors back into HBM (serving only)."""
        from .. import persistence
        _, uids, U, pids, V = persistence.load_mllib(path)
        return cls(_engine.ALSCore.from_factors(uids, U.astype(np.float32), pids,
                                                V.astype(np.float32)))

    def recommendUsersForProducts(self, num: int):
        keys, ids, sc = self._core.recommend_all(int(num), False)
        keys, ids, sc = keys.cpu().numpy(), ids.cpu().numpy(), sc.cpu().numpy()
        return [(int(k), [Rating(int(a), int(k), float(s)) for a, s in zip(ri, rs)
                          if np.isfinite(s)])
                for k, ri, rs in zip(keys, ids, sc)]


def _check(rank, iterations, lambda_, nonnegative, alpha=0.0):
    if int(rank) < 1:
        raise ValueError(f"rank must be >= 1, got {rank}")
    if int(rank) > 128:
        raise NotImplementedError("rank > 128 is not supported by this build of the HIP kernels")
    if int(iterations) < 0:
        raise ValueError(f"iterations must be >= 0, got {iterations}")
    if lambda_ < 0:
        raise ValueError(f"lambda_ must be >= 0, got {lambda_}")
    if alpha < 0:
        raise ValueError(f"alpha must be >= 0, got {alpha}")
    if nonnegative:
        raise NotImplementedError("nonnegative=True (NNLS solver) is out of scope for this build")


class ALS:
    """Alternating Least Squares matrix factorisation (pyspark.mllib API)."""

    @classmethod
    def train(cls, ratings, rank: int, iterations: int = 5, lambda_: float = 0.01,
              blocks: int = -1, nonnegative: bool = False, seed: Optional[int] = None
              ) -> MatrixFactorizationModel:
        _check(rank, iterations, lambda_, nonnegative)
        u, i, r = _triples(ratings)
        core = _engine.make_engine(u, i, r)
        core.fit(int(rank), int(iterations), float(lambda_), False, 1.0,
                 seed=_DEFAULT_SEED if seed is None else int(seed))
        return MatrixFactorizationModel(core)

    @classmethod
    def trainImplicit(cls, ratings, rank: int, iterations: int = 5, lambda_: float = 0.01,
                      blocks: int = -1, alpha: float = 0.01, nonnegative: bool = False,
                      seed: Optional[int] = None) -> MatrixFactorizationModel:
        _check(rank, iterations, lambda_, nonnegative, alpha)
        u, i, r = _triples(ratings)
        core = _engine.make_engine(u, i, r)
        core.fit(int(rank), int(iterations), float(lambda_), True, float(alpha),
                 seed=_DEFAULT_SEED if seed is None else int(seed))
        return MatrixFactorizationModel(core)


def compute_error(predicted: Iterable, actual: Iterable) -> float:
    """RecommenderSystem.py:103-129 computeError as host glue over predictAll output:
    join on (user, product), sqrt(mean squared error).  (Use
    MatrixFactorizationModel.rmse for the fused on-device form.)"""
    import math
    pred = {}
    for u, i, r in predicted:
        pred.setdefault((int(u), int(i)), []).append(float(r))
    total, n = 0.0, 0
    for u, i, r in actual:
        for p in pred.get((int(u), int(i)), ()):
            total += (float(r) - p) ** 2
            n += 1
    return math.sqrt(total / n)
