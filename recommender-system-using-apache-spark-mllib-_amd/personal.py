"""The reference's personal-recommendation flow as a host helper over K4.

RecommenderSystem.py:227-249, restated for the MI355X engine:

  R:229  myUnratedMoviesRDD  = every (user, MovieID) of moviesRDD the user has not rated
  R:232  predictAll(...)     -> K4 als_predict on the device (inner join: movies the
                                model has never seen are dropped, as Spark's join does)
  R:236  movieCountsRDD      = (MovieID, number of ratings) from getCountsAndAverages
  R:242-245 join with counts and titles, keep NumRating > 75
  R:247  takeOrdered(20, key=-prediction)

`movie_counts_and_averages` is R:50-58's getCountsAndAverages over the full ratings
(the count the R:245 filter reads).  Ties in the prediction keep moviesRDD order
(takeOrdered is heapq.nsmallest over the partitions: stable for equal keys).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple

import numpy as np

__all__ = ["movie_counts_and_averages", "personal_recommendations"]


def movie_counts_and_averages(ratings) -> Dict[int, Tuple[int, float]]:
    """R:50-58 getCountsAndAverages over (user, movie, rating) triples:
    MovieID -> (number of ratings, average rating)."""
    from ._data import columns_of
    _, m, r = columns_of(ratings, ("user", "movie", "rating"))
    m = np.asarray(m, np.int64)
    r = np.asarray(r, np.float64)
    ids, inv, cnt = np.unique(m, return_inverse=True, return_counts=True)
    tot = np.bincount(inv, weights=r)
    return {int(a): (int(c), float(t) / int(c)) for a, c, t in zip(ids, cnt, tot)}


def _engine_of(model):
    eng = getattr(model, "engine", None)
    if eng is None:
        raise TypeError("expected a MatrixFactorizationModel or ALSModel")
    return eng


def personal_recommendations(model, user_id: int, rated: Iterable[Sequence],
                             movies: Iterable[Sequence], counts, min_count: int = 75,
                             num: int = 20) -> List[Tuple[float, str, int]]:
    """(predicted rating, movie name, number of ratings) for the user's top `num`
    unrated movies with more than `min_count` ratings, highest prediction first.

    rated:  the user's (user, movie, rating) triples (myRatedMovies, R:190-202)
    movies: (MovieID, title) pairs (moviesRDD, R:39)
    counts: MovieID -> number of ratings, or MovieID -> (count, average) as
            returned by movie_counts_and_averages (movieCountsRDD, R:236)."""
    rated_pairs = {(int(u), int(m)) for u, m, *_ in rated}
    movies = [(int(m), str(t)) for m, t in movies]
    cand = [(m, t) for m, t in movies if (int(user_id), m) not in rated_pairs]   # R:229
    if not cand:
        return []
    mids = np.fromiter((m for m, _ in cand), dtype=np.int64, count=len(cand))
    ok_range = (mids >= -(2 ** 31)) & (mids < 2 ** 31)
    pred = np.full(len(cand), np.nan)
    users = np.full(int(ok_range.sum()), int(user_id), np.int32)
    pred[ok_range] = _engine_of(model).predict(users, mids[ok_range].astype(np.int32)
                                               ).cpu().numpy()                  # R:232
    out = []
    for (m, title), p in zip(cand, pred):
        if np.isnan(p):           # predictAll's inner join drops unknown movies
            continue
        c = counts.get(m)         # R:242 join with movieCountsRDD
        if c is None:
            continue
        n = int(c[0]) if isinstance(c, tuple) else int(c)
        if n > min_count:         # R:245
            out.append((float(p), title, n))
    # R:247 takeOrdered(num, key=-rating): stable for equal predictions
    order = sorted(range(len(out)), key=lambda j: -out[j][0])
    return [out[j] for j in order[:num]]
