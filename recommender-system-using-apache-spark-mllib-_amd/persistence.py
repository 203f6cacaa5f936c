"""Model persistence in Spark's on-disk layout.

Upstream (not vendored; restated): ``MatrixFactorizationModel.SaveLoadV1_0``
(mllib/recommendation/MatrixFactorizationModel.scala) writes

    <path>/metadata/part-00000          one JSON line: {"class": ..., "version": "1.0", "rank": k}
    <path>/data/user/part-00000.parquet    columns id: int32, features: list<double>
    <path>/data/product/part-00000.parquet columns id: int32, features: list<double>

and ``ALSModel`` (ml/recommendation/ALS.scala, ``ALSModelWriter``) writes

    <path>/metadata/part-00000          JSON: class, timestamp, sparkVersion, uid, paramMap, rank
    <path>/userFactors/part-00000.parquet  columns id: int32, features: list<float>
    <path>/itemFactors/part-00000.parquet  columns id: int32, features: list<float>

This module reads and writes those files with pyarrow (host arrays in, host
arrays out).  Factors are stored at the precision each format names (fp64 for
mllib, fp32 for ml), so an fp32 factor table round-trips bit-exactly through
either.
"""
from __future__ import annotations

import json
import os
import shutil
import time
from typing import Dict, Tuple

import numpy as np

MLLIB_CLASS = "org.apache.spark.mllib.recommendation.MatrixFactorizationModel"
ML_CLASS = "org.apache.spark.ml.recommendation.ALSModel"
FORMAT_VERSION = "1.0"
# DefaultParamsReader parses sparkVersion with VersionUtils.majorMinorVersion and,
# from 2.4 on, expects a defaultParamMap next to paramMap.
SPARK_VERSION = "3.5.0"
# ALSModel's own params (ALSModelParams) and their defaults: the only keys
# DefaultParamsWriter records for the model.
ML_MODEL_DEFAULTS = {"blockSize": 4096, "coldStartStrategy": "nan", "itemCol": "item",
                     "predictionCol": "prediction", "userCol": "user"}


def _pa():
    try:
        import pyarrow as pa
        import pyarrow.parquet as pq
    except ImportError as e:  # pragma: no cover - pyarrow ships in this image
        raise RuntimeError("model persistence needs pyarrow (Spark stores factors as Parquet)") from e
    return pa, pq


def _write_factors(path: str, ids, F, np_dtype, value_type) -> None:
    pa, pq = _pa()
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    F = np.ascontiguousarray(F, dtype=np_dtype)
    if F.ndim != 2 or F.shape[0] != ids.shape[0]:
        raise ValueError(f"factor table {F.shape} does not match {ids.shape[0]} ids")
    k = F.shape[1]
    flat = pa.array(F.reshape(-1), type=value_type)
    offsets = pa.array(np.arange(0, (len(ids) + 1) * k, k, dtype=np.int32), type=pa.int32())
    feats = pa.ListArray.from_arrays(offsets, flat)
    table = pa.table({"id": pa.array(ids, type=pa.int32()), "features": feats})
    os.makedirs(path, exist_ok=True)
    pq.write_table(table, os.path.join(path, "part-00000.parquet"))
    open(os.path.join(path, "_SUCCESS"), "w").close()


def _read_factors(path: str, rank: int, dtype) -> Tuple[np.ndarray, np.ndarray]:
    _, pq = _pa()
    files = sorted(f for f in os.listdir(path) if f.endswith(".parquet"))
    if not files:
        raise FileNotFoundError(f"no parquet part files under {path}")
    ids, feats = [], []
    for f in files:
        t = pq.read_table(os.path.join(path, f), columns=["id", "features"])
        ids.append(t.column("id").to_numpy().astype(np.int32))
        col = t.column("features").combine_chunks()
        lens = np.diff(col.offsets.to_numpy())
        if len(lens) and (lens != rank).any():
            raise ValueError(f"{path}: feature vectors of length {sorted(set(lens.tolist()))}, "
                             f"expected rank {rank}")
        vals = col.values.to_numpy(zero_copy_only=False)
        feats.append(np.asarray(vals, dtype=dtype).reshape(-1, rank))
    ids = np.concatenate(ids)
    F = np.concatenate(feats)
    order = np.argsort(ids, kind="stable")  # part files need not be id-ordered
    ids, F = ids[order], F[order]
    if len(ids) > 1 and (np.diff(ids) == 0).any():
        raise ValueError(f"{path}: duplicate ids")
    return ids, F


def _write_metadata(path: str, meta: Dict) -> None:
    d = os.path.join(path, "metadata")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "part-00000"), "w") as f:
        f.write(json.dumps(meta, separators=(",", ":")) + "\n")
    open(os.path.join(d, "_SUCCESS"), "w").close()


def _read_metadata(path: str) -> Dict:
    d = os.path.join(path, "metadata")
    parts = sorted(f for f in os.listdir(d) if f.startswith("part-"))
    if not parts:
        raise FileNotFoundError(f"no metadata part file under {d}")
    with open(os.path.join(d, parts[0])) as f:
        return json.loads(f.readline())


def _check_target(path: str, overwrite: bool) -> None:
    """Spark: "Path ... already exists" unless write.overwrite(), which deletes the
    path first (stale part files must not be read back with the new ones)."""
    if os.path.lexists(path):
        if not overwrite and (not os.path.isdir(path) or os.listdir(path)):
            raise FileExistsError(f"Path {path} already exists")
        if overwrite:
            if os.path.isdir(path) and not os.path.islink(path):
                shutil.rmtree(path)
            else:
                os.remove(path)


def save_mllib(path: str, rank: int, user_ids, U, product_ids, V, overwrite: bool = False) -> None:
    """MatrixFactorizationModel.save(sc, path): metadata + data/user + data/product (fp64)."""
    _check_target(path, overwrite)
    pa, _ = _pa()
    _write_metadata(path, {"class": MLLIB_CLASS, "version": FORMAT_VERSION, "rank": int(rank)})
    _write_factors(os.path.join(path, "data", "user"), user_ids, U, np.float64, pa.float64())
    _write_factors(os.path.join(path, "data", "product"), product_ids, V, np.float64, pa.float64())


def load_mllib(path: str):
    """MatrixFactorizationModel.load(sc, path) -> (rank, user_ids, U, product_ids, V), host fp64."""
    meta = _read_metadata(path)
    if meta.get("class") != MLLIB_CLASS or meta.get("version") != FORMAT_VERSION:
        raise ValueError(f"{path}: not a {MLLIB_CLASS} v{FORMAT_VERSION} model "
                         f"(class={meta.get('class')}, version={meta.get('version')})")
    rank = int(meta["rank"])
    uids, U = _read_factors(os.path.join(path, "data", "user"), rank, np.float64)
    pids, V = _read_factors(os.path.join(path, "data", "product"), rank, np.float64)
    return rank, uids, U, pids, V


def save_ml(path: str, uid: str, params: Dict, rank: int, user_ids, U, item_ids, V,
            overwrite: bool = False) -> None:
    """ALSModel.write.save(path): metadata (paramMap of the set model params,
    defaultParamMap) + userFactors + itemFactors (fp32)."""
    _check_target(path, overwrite)
    pa, _ = _pa()
    set_params = {k: v for k, v in params.items() if k in ML_MODEL_DEFAULTS}
    _write_metadata(path, {"class": ML_CLASS, "timestamp": int(time.time() * 1000),
                           "sparkVersion": SPARK_VERSION, "uid": uid, "paramMap": set_params,
                           "defaultParamMap": dict(ML_MODEL_DEFAULTS), "rank": int(rank)})
    _write_factors(os.path.join(path, "userFactors"), user_ids, U, np.float32, pa.float32())
    _write_factors(os.path.join(path, "itemFactors"), item_ids, V, np.float32, pa.float32())


def load_ml(path: str):
    """ALSModel.load(path) -> (uid, params, rank, user_ids, U, item_ids, V), host fp32."""
    meta = _read_metadata(path)
    if meta.get("class") != ML_CLASS:
        raise ValueError(f"{path}: not an {ML_CLASS} (class={meta.get('class')})")
    rank = int(meta["rank"])
    uids, U = _read_factors(os.path.join(path, "userFactors"), rank, np.float32)
    iids, V = _read_factors(os.path.join(path, "itemFactors"), rank, np.float32)
    return meta.get("uid"), meta.get("paramMap", {}), rank, uids, U, iids, V
