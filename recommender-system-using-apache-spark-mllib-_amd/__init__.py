"""als_mi355x — MI355X-native drop-in for the ALS hot path of
amy-leaf/Recommender-System-using-Apache-Spark-MLlib-.

Import name: ``als_mi355x`` (this directory is registered under that name by
``_pkgload.load()`` at the repository root, because the directory name itself is
not a Python identifier).

Surfaces (mirroring pyspark's module layout):
  als_mi355x.ml.recommendation     ALS, ALSModel           (pyspark.ml.recommendation)
  als_mi355x.mllib.recommendation  ALS, MatrixFactorizationModel, Rating
                                                           (pyspark.mllib.recommendation,
                                                            RecommenderSystem.py:132)
  als_mi355x.engine                ALSCore — the device-resident engine
  als_mi355x.distributed           one-process-per-GPU sharded ALS (RCCL all-gather)
"""
__version__ = "0.1.0"

from . import _lib  # noqa: F401
