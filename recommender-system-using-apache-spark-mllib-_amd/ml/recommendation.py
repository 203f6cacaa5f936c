"""pyspark.ml.recommendation-compatible surface: ALS (estimator) and ALSModel.

Drop-in for the north-star API of the reference's ALS path
(``pyspark.ml.recommendation.ALS(rank, maxIter, regParam, implicitPrefs,
alpha, coldStartStrategy, ...)`` with ``fit()`` / ``transform()`` /
``recommendForAllUsers()``), backed by the MI355X engine (als_mi355x.engine).
Datasets are pandas DataFrames (or dicts of arrays) instead of Spark
DataFrames; column names, parameter names, defaults and error conditions
follow Spark's ``ALSParams`` (ml/recommendation/ALS.scala, upstream).
"""
from __future__ import annotations

import zlib
from typing import Optional

import numpy as np
import torch

from .. import engine as _engine
from .._data import check_integers, columns_of, to_float32

__all__ = ["ALS", "ALSModel"]

_DEFAULT_SEED = zlib.crc32(b"org.apache.spark.ml.recommendation.ALS")
_COLD = ("nan", "drop")


def _validate(p: dict) -> None:
    """ALSParams validators (ParamValidators.gtEq / inArray), IllegalArgumentException -> ValueError."""
    if not isinstance(p["rank"], (int, np.integer)) or p["rank"] < 1:
        raise ValueError(f"ALS_rank parameter rank given invalid value {p['rank']} (must be >= 1)")
    if not isinstance(p["maxIter"], (int, np.integer)) or p["maxIter"] < 0:
        raise ValueError(f"ALS_maxIter parameter maxIter given invalid value {p['maxIter']}")
    if p["regParam"] < 0:
        raise ValueError(f"ALS_regParam parameter regParam given invalid value {p['regParam']}")
    if p["alpha"] < 0:
        raise ValueError(f"ALS_alpha parameter alpha given invalid value {p['alpha']}")
    if p["numUserBlocks"] < 1 or p["numItemBlocks"] < 1:
        raise ValueError("numUserBlocks/numItemBlocks must be >= 1")
    if p["checkpointInterval"] < 1 and p["checkpointInterval"] != -1:
        raise ValueError("checkpointInterval must be -1 or >= 1")
    if str(p["coldStartStrategy"]).lower() not in _COLD:
        raise ValueError(f"ALS_coldStartStrategy parameter coldStartStrategy given invalid value "
                         f"{p['coldStartStrategy']} (supported: {', '.join(_COLD)})")
    if p["rank"] > 128:
        raise NotImplementedError("rank > 128 is not supported by this build of the HIP kernels")
    if p["nonnegative"]:
        raise NotImplementedError("nonnegative=True (NNLS solver) is out of scope for this build")


class _Params:
    _defaults = dict(rank=10, maxIter=10, regParam=0.1, numUserBlocks=10, numItemBlocks=10,
                     implicitPrefs=False, alpha=1.0, userCol="user", itemCol="item", seed=None,
                     ratingCol="rating", nonnegative=False, checkpointInterval=10,
                     intermediateStorageLevel="MEMORY_AND_DISK",
                     finalStorageLevel="MEMORY_AND_DISK", coldStartStrategy="nan",
                     blockSize=4096, predictionCol="prediction")

    def _init_params(self, kw):
        unknown = set(kw) - set(self._defaults)
        if unknown:
            raise TypeError(f"unexpected keyword argument(s): {sorted(unknown)}")
        self._p = dict(self._defaults)
        self._p.update(kw)

    def getOrDefault(self, name):
        return self._p[name]


def _make_accessors(cls, names):
    for n in names:
        cap = n[0].upper() + n[1:]

        def setter(self, value, _n=n):
            self._p[_n] = value
            return self

        def getter(self, _n=n):
            return self._p[_n]

        setattr(cls, "set" + cap, setter)
        setattr(cls, "get" + cap, getter)


class ALS(_Params):
    """Alternating Least Squares (explicit or implicit feedback) on one MI355X.

    ``numUserBlocks`` / ``numItemBlocks`` / storage levels are accepted for signature
    compatibility and have no effect (the ratings are a single device-resident CSR
    per side).  ``checkpointInterval`` acts as in Spark once a checkpoint directory
    is set (``setCheckpointDir``, the role of ``SparkContext.setCheckpointDir``):
    the factors are written every ``checkpointInterval`` iterations, and a fit of
    the same ratings and params in that directory resumes from the checkpoint
    (checkpoint.py) instead of starting over.
    """

    def __init__(self, **kw):
        self._init_params(kw)
        self._checkpoint_dir = None

    def setCheckpointDir(self, path):
        """Directory for factor checkpoints (None disables)."""
        self._checkpoint_dir = None if path is None else str(path)
        return self

    def setParams(self, **kw):
        for k, v in kw.items():
            if k not in self._defaults:
                raise TypeError(f"unknown parameter {k}")
            self._p[k] = v
        return self

    def setNumBlocks(self, value):
        self._p["numUserBlocks"] = value
        self._p["numItemBlocks"] = value
        return self

    def fit(self, dataset) -> "ALSModel":
        p = self._p
        _validate(p)
        u, i, r = columns_of(dataset, (p["userCol"], p["itemCol"], p["ratingCol"]))
        u = check_integers(u, p["userCol"])
        i = check_integers(i, p["itemCol"])
        r = to_float32(r)
        seed = _DEFAULT_SEED if p["seed"] is None else int(p["seed"])
        core = _engine.make_engine(u, i, r)
        core.fit(int(p["rank"]), int(p["maxIter"]), float(p["regParam"]),
                 bool(p["implicitPrefs"]), float(p["alpha"]), seed=seed,
                 checkpoint_dir=self._checkpoint_dir,
                 checkpoint_interval=int(p["checkpointInterval"]), resume="auto")
        return ALSModel(core, dict(p))


_make_accessors(ALS, list(_Params._defaults))


class ALSModel:
    """Fitted factors resident in HBM; mirrors pyspark.ml.recommendation.ALSModel."""

    def __init__(self, core: "_engine.ALSCore", params: dict):
        self._core = core
        self._p = params

    # -- params used at transform time --
    def setUserCol(self, v):
        self._p["userCol"] = v
        return self

    def setItemCol(self, v):
        self._p["itemCol"] = v
        return self

    def setPredictionCol(self, v):
        self._p["predictionCol"] = v
        return self

    def setColdStartStrategy(self, v):
        if str(v).lower() not in _COLD:
            raise ValueError(f"ALS_coldStartStrategy parameter coldStartStrategy given invalid "
                             f"value {v} (supported: {', '.join(_COLD)})")
        self._p["coldStartStrategy"] = v
        return self

    def setBlockSize(self, v):
        self._p["blockSize"] = v
        return self

    @property
    def rank(self) -> int:
        return self._core.rank

    @property
    def engine(self) -> "_engine.ALSCore":
        return self._core

    def _factors_df(self, ids, F):
        import pandas as pd
        ids = ids.cpu().numpy()
        F = F.float().cpu().numpy()
        return pd.DataFrame({"id": ids, "features": list(F)})

    def save(self, path: str, overwrite: bool = False) -> None:
        """ALSModel.save(path) / write().save(path) in Spark's layout."""
        from .. import persistence
        uids, U = self._core.user_factors()
        iids, V = self._core.item_factors()
        params = {k: v for k, v in self._p.items() if isinstance(v, (int, float, str, bool))}
        persistence.save_ml(path, "ALSModel_mi355x", params, self.rank, uids.cpu().numpy(),
                            U.cpu().numpy(), iids.cpu().numpy(), V.cpu().numpy(),
                            overwrite=overwrite)

    @classmethod
    def load(cls, path: str) -> "ALSModel":
        """ALSModel.load(path): factors back into HBM (serving only), params restored."""
        from .. import persistence
        _, params, _, uids, U, iids, V = persistence.load_ml(path)
        p = dict(_Params._defaults)
        p.update({k: v for k, v in params.items() if k in p})
        return cls(_engine.ALSCore.from_factors(uids, U, iids, V), p)

    @property
    def userFactors(self):
        return self._factors_df(*self._core.user_factors())

    @property
    def itemFactors(self):
        return self._factors_df(*self._core.item_factors())

    def transform(self, dataset):
        """Append the prediction column (fp32 <u, v>; NaN for unknown ids, or those rows
        dropped when coldStartStrategy == "drop")."""
        import pandas as pd
        p = self._p
        u, i = columns_of(dataset, (p["userCol"], p["itemCol"]))
        u = check_integers(u, p["userCol"])
        i = check_integers(i, p["itemCol"])
        pred = self._core.predict(u, i).float().cpu().numpy()
        if isinstance(dataset, pd.DataFrame):
            out = dataset.copy()
        else:
            out = pd.DataFrame({p["userCol"]: u, p["itemCol"]: i})
        out[p["predictionCol"]] = pred
        if str(p["coldStartStrategy"]).lower() == "drop":
            out = out[~np.isnan(pred)]
        return out

    def rmse(self, dataset, ratingCol: Optional[str] = None) -> float:
        """RMSE over rows whose user and item are known (fused gather-dot-reduce, K4) —
        the device form of RecommenderSystem.py:103-129's computeError."""
        p = self._p
        u, i, r = columns_of(dataset, (p["userCol"], p["itemCol"], ratingCol or p["ratingCol"]))
        rm, _ = self._core.rmse(check_integers(u, p["userCol"]), check_integers(i, p["itemCol"]),
                                to_float32(r))
        return rm

    # -- recommendForAll (K5) --
    def recommendForAllUsersArrays(self, numItems: int):
        """Device tensors (user ids [n_u], item ids [n_u, t], scores [n_u, t]),
        t = min(numItems, n_items).  Multi-GPU: this rank's users (its partition)."""
        return self._core.recommend_all(int(numItems), True)

    def recommendForAllItemsArrays(self, numUsers: int):
        return self._core.recommend_all(int(numUsers), False)

    @staticmethod
    def _recs_df(key_col, keys, ids, sc):
        import pandas as pd
        keys = keys.cpu().numpy()
        ids = ids.cpu().numpy()
        sc = sc.cpu().numpy()
        # empty slots (score -inf: a query row whose every score is NaN) are dropped
        recs = [[(int(a), float(b)) for a, b in zip(ri, rs) if np.isfinite(b)]
                for ri, rs in zip(ids, sc)]
        return pd.DataFrame({key_col: keys, "recommendations": recs})

    def recommendForAllUsers(self, numItems: int):
        """DataFrame[userCol, recommendations: list of (item, rating)], rating desc
        (ties: lower item id first)."""
        return self._recs_df(self._p["userCol"], *self.recommendForAllUsersArrays(numItems))

    def recommendForAllItems(self, numUsers: int):
        return self._recs_df(self._p["itemCol"], *self.recommendForAllItemsArrays(numUsers))

    def recommendForUserSubset(self, dataset, numItems: int):
        """Top items for the distinct known users of `dataset[userCol]`."""
        col = self._p["userCol"]
        ids = check_integers(columns_of(dataset, (col,))[0], col)
        return self._recs_df(col, *self._core.recommend_subset(ids, int(numItems), True))

    def recommendForItemSubset(self, dataset, numUsers: int):
        col = self._p["itemCol"]
        ids = check_integers(columns_of(dataset, (col,))[0], col)
        return self._recs_df(col, *self._core.recommend_subset(ids, int(numUsers), False))
