"""Host-side argument handling shared by the ml and mllib surfaces.

Mirrors Spark's input checks for the ALS path:
  * ALS.checkIntegers (ml/recommendation/ALS.scala, upstream): user/item
    columns must hold integer values inside the Int range, else
    IllegalArgumentException -> here ValueError with Spark's wording;
  * ratings are cast to Float (mllib ALS.run: `r.rating.toFloat`).
"""
from __future__ import annotations

from typing import Any, Tuple

import numpy as np

INT_MIN, INT_MAX = -(2 ** 31), 2 ** 31 - 1


def check_integers(values: np.ndarray, col: str) -> np.ndarray:
    v = np.asarray(values)
    if v.dtype.kind in "iu":
        if v.size and (v.min() < INT_MIN or v.max() > INT_MAX):
            raise ValueError(f"ALS only supports values in Integer range for column {col}. "
                             f"Value {v.max() if v.max() > INT_MAX else v.min()} was out of "
                             "Integer range.")
        return v.astype(np.int32)
    if v.dtype.kind == "f":
        bad = ~np.isfinite(v) | (v != np.round(v)) | (v < INT_MIN) | (v > INT_MAX)
        if v.size and bad.any():
            x = v[np.argmax(bad)]
            raise ValueError(f"ALS only supports values in Integer range and without fractional "
                             f"part for column {col}. Value {x} was either out of Integer range "
                             "or contained a fractional part that could not be converted.")
        return v.astype(np.int32)
    if v.dtype == object:
        return check_integers(np.asarray(v.tolist(), dtype=np.float64), col)
    raise ValueError(f"column {col} must be numeric, got dtype {v.dtype}")


def to_float32(values) -> np.ndarray:
    return np.asarray(values, dtype=np.float64).astype(np.float32)


def columns_of(dataset: Any, cols: Tuple[str, ...]):
    """Extract named columns from a pandas DataFrame, dict of arrays or numpy
    structured array; a (n, len(cols)) array / list of tuples is taken positionally."""
    try:
        import pandas as pd
        if isinstance(dataset, pd.DataFrame):
            missing = [c for c in cols if c not in dataset.columns]
            if missing:
                raise ValueError(f"dataset has no column(s) {missing}; columns: "
                                 f"{list(dataset.columns)}")
            return [dataset[c].to_numpy() for c in cols]
    except ImportError:  # pragma: no cover
        pass
    if isinstance(dataset, dict):
        return [np.asarray(dataset[c]) for c in cols]
    if isinstance(dataset, np.ndarray) and dataset.dtype.names:
        return [dataset[c] for c in cols]
    try:
        import torch
        if isinstance(dataset, torch.Tensor):
            dataset = dataset.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    arr = np.asarray(list(dataset) if not isinstance(dataset, np.ndarray) else dataset,
                     dtype=np.float64)
    if arr.ndim != 2 or arr.shape[1] < len(cols):
        raise ValueError(f"expected rows of {len(cols)} values ({', '.join(cols)})")
    return [arr[:, j] for j in range(len(cols))]
