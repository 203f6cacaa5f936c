"""Rating sources for the ALS path: MovieLens-format parsers and the seeded
synthetic generators the benchmarks use.

Parsers restate RecommenderSystem.py:16-35 (``get_ratings_tuple``: the
``UserID::MovieID::Rating::Timestamp`` line -> (int, int, float), timestamp
dropped; ``get_movie_tuple``: ``MovieID::Title::Genres`` -> (int, str)), read
``.gz`` transparently, and also accept the ml-latest / ml-25m CSV layout.

The synthetic generator runs on the device with torch (data plumbing, not the
product's arithmetic): planted low-rank ratings
``clip(round_half(mu + <u*, v*> + eps), 0.5, 5)``, k_true = 16, u*, v* ~ N(0, 0.35^2),
mu = 3.6, eps ~ N(0, 0.8^2); log-normal user degrees (min 20); Zipf(0.9) item
popularity capped at half the users; no duplicate (user, item) pairs.
"""
from __future__ import annotations

import gzip
import io
import math
from typing import Tuple

import numpy as np
import torch


# ---------------------------------------------------------------- parsers
def get_ratings_tuple(entry: str):
    """RecommenderSystem.py:16-24."""
    items = entry.split("::")
    return int(items[0]), int(items[1]), float(items[2])


def get_movie_tuple(entry: str):
    """RecommenderSystem.py:27-35."""
    items = entry.split("::")
    return int(items[0]), items[1]


def _open_text(path: str):
    if path.endswith(".gz"):
        return io.TextIOWrapper(gzip.open(path, "rb"), encoding="utf-8", errors="replace")
    return open(path, "r", encoding="utf-8", errors="replace")


def load_ratings(path: str) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """ratings.dat[.gz] ('::' separated) or ratings.csv (userId,movieId,rating,timestamp)
    -> (users int32, items int32, ratings float32), file order."""
    users, items, vals = [], [], []
    with _open_text(path) as f:
        first = f.readline()
        sep = "::" if "::" in first else ","
        lines = [first] if (sep == "::" or first[:1].isdigit()) else []
        for line in lines + list(f):
            line = line.strip()
            if not line:
                continue
            p = line.split(sep)
            users.append(int(p[0]))
            items.append(int(p[1]))
            vals.append(float(p[2]))
    return (np.asarray(users, np.int32), np.asarray(items, np.int32),
            np.asarray(vals, np.float32))


def load_movies(path: str):
    """movies.dat ('::') or movies.csv -> list of (MovieID, Title)."""
    out = []
    with _open_text(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line or line.startswith("movieId"):
                continue
            if "::" in line:
                out.append(get_movie_tuple(line))
            else:  # csv: movieId,title,genres (title may be quoted)
                mid, rest = line.split(",", 1)
                title = rest.rsplit(",", 1)[0].strip('"')
                out.append((int(mid), title))
    return out


def random_split(n: int, weights=(6, 2, 2), seed: int = 0):
    """Seeded split into len(weights) index sets with the given proportions (the
    role of RDD.randomSplit at RecommenderSystem.py:90; Spark's sampler RNG itself is
    not reproduced)."""
    w = np.asarray(weights, np.float64)
    cut = np.cumsum(w / w.sum())
    x = np.random.default_rng(seed).random(n)
    bins = np.searchsorted(cut, x, side="right")
    return [np.nonzero(bins == b)[0] for b in range(len(weights))]


# ---------------------------------------------------------------- synthetic
CONFIGS = {
    # name: (n_users, n_items, nnz, half_stars, data_seed)
    "ml1m_lab4": (6040, 3706, 292716, False, 0),        # SURVEY 0a (script-as-written)
    "ml_latest_small": (610, 9724, 100836, True, 0),    # SURVEY 0b (BASELINE configs[0])
    "ml25m": (162541, 59047, 25000095, True, 1),         # BASELINE configs[1] / [2]
    "big1b": (10_000_000, 1_000_000, 1_000_000_000, True, 2),  # BASELINE configs[3] / [4]
}


def _zipf_probs(n_items: int, s: float, cap: float) -> torch.Tensor:
    p = 1.0 / torch.arange(1, n_items + 1, dtype=torch.float64) ** s
    p /= p.sum()
    for _ in range(50):  # water-fill the cap
        over = p > cap
        if not over.any():
            break
        excess = (p[over] - cap).sum()
        p[over] = cap
        p[~over] += excess * p[~over] / p[~over].sum()
    return p


def synthetic(n_users: int, n_items: int, nnz: int, seed: int = 1, half_stars: bool = True,
              device="cuda", k_true: int = 16, user_offset: int = 0, users_total: int = None
              ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Seeded planted-model ratings on `device`: (users int32, items int32, ratings f32),
    exactly `nnz` distinct (user, item) pairs.  `user_offset` / `users_total` let ranks
    of a sharded job generate disjoint user ranges of one global dataset."""
    dev = torch.device(device)
    g = torch.Generator(device="cpu")
    g.manual_seed(seed * 1000003 + user_offset)
    if nnz > n_users * n_items // 2:
        raise ValueError("synthetic: too dense for rejection sampling")
    # user degrees: log-normal, min 20, rescaled to sum to nnz
    deg = torch.exp(torch.randn(n_users, generator=g, dtype=torch.float64) * 1.0 + 4.2)
    deg = 20 + deg * max(nnz - 20 * n_users, 0) / deg.sum()
    deg = deg.clamp(max=n_items * 0.5)
    d = torch.floor(deg).long()
    short = nnz - int(d.sum())
    if short > 0:
        frac = deg - d
        cf = torch.cumsum(frac, 0)
        add = torch.searchsorted(cf / cf[-1], torch.rand(short, generator=g, dtype=torch.float64))
        d += torch.bincount(add.clamp(max=n_users - 1), minlength=n_users)
    pop = _zipf_probs(n_items, 0.9, 0.5 * n_users / nnz).to(torch.float32)
    gi = torch.Generator(device="cpu")
    gi.manual_seed(seed * 15485863)  # item id permutation shared by every user shard
    perm_items = torch.randperm(n_items, generator=gi)  # popular items scattered over ids
    gd = torch.Generator(device=dev)
    gd.manual_seed(seed * 7919 + user_offset)
    pop_d = pop.to(dev)
    users = torch.repeat_interleave(torch.arange(n_users, device=dev), d.to(dev))
    keys = torch.empty(0, dtype=torch.int64, device=dev)
    want = users
    cdf_i = torch.cumsum(pop_d.double(), 0)
    cdf_i = (cdf_i / cdf_i[-1]).float()
    cdf_u = torch.cumsum(d.double(), 0).to(dev)
    cdf_u = (cdf_u / cdf_u[-1]).float()
    for _ in range(64):
        x = torch.rand(want.numel(), generator=gd, device=dev)
        it = torch.searchsorted(cdf_i, x).clamp(max=n_items - 1)
        keys = torch.unique(torch.cat([keys, want * n_items + it]))
        missing = nnz - keys.numel()
        if missing <= 0:
            break
        # top up with users drawn proportional to degree
        x = torch.rand(missing + missing // 8 + 16, generator=gd, device=dev)
        want = torch.searchsorted(cdf_u, x).clamp(max=n_users - 1)
    if keys.numel() < nnz:
        raise RuntimeError("synthetic generator failed to reach nnz")
    if keys.numel() > nnz:
        keep = torch.randperm(keys.numel(), generator=gd, device=dev)[:nnz]
        keys = keys[torch.sort(keep).values]
    u = keys // n_items
    i = perm_items.to(dev)[keys % n_items]
    # planted model
    us = torch.randn((n_users, k_true), generator=gd, device=dev) * 0.35
    vs_g = torch.Generator(device=dev)
    vs_g.manual_seed(seed * 104729)  # item factors shared by all user shards
    vs = torch.randn((n_items, k_true), generator=vs_g, device=dev) * 0.35
    r = torch.empty(nnz, dtype=torch.float32, device=dev)
    step = 1 << 22
    for s in range(0, nnz, step):
        e = min(nnz, s + step)
        dot = (us[u[s:e]] * vs[i[s:e]]).sum(1)
        x = 3.6 + dot + 0.8 * torch.randn(e - s, generator=gd, device=dev)
        if half_stars:
            r[s:e] = (torch.round(x * 2) / 2).clamp(0.5, 5.0)
        else:
            r[s:e] = torch.round(x).clamp(1.0, 5.0)
    # shuffle rating order (input order must not be pre-sorted)
    perm = torch.randperm(nnz, generator=gd, device=dev)
    return ((u[perm] + user_offset).to(torch.int32), i[perm].to(torch.int32), r[perm])


def synthetic_config(name: str, device="cuda", scale_users: int = 1, shard: int = 0):
    """One of CONFIGS; `scale_users` replicates the user population (weak scaling:
    shard s of S holds users [s*n_u, (s+1)*n_u) and nnz ratings)."""
    n_u, n_i, nnz, half, seed = CONFIGS[name]
    return synthetic(n_u, n_i, nnz, seed=seed, half_stars=half, device=device,
                     user_offset=shard * n_u)


# ---------------------------------------------------------------- 1B-rating power law
def synthetic_blocked(n_users: int, n_items: int, nnz: int, seed: int = 2, half_stars: bool = True,
                      device="cuda", user_begin: int = 0, user_end: int = None,
                      block_ratings: int = 1 << 26, k_true: int = 16):
    """BASELINE configs[3]: the planted model of `synthetic` at 1e9-rating scale,
    generated on the device in user blocks (never the whole key set at once).

    Users [user_begin, user_end) of one global dataset are produced, so ranks of a
    sharded job generate disjoint user ranges whose union is exactly the
    single-process dataset (every quantity is derived from `seed` and the global
    user index).  Degrees: log-normal (min 20) scaled to `nnz` over ALL users;
    items: Zipf(0.9) popularity capped at half the users (SURVEY.md §8d caps the
    head item at n_users).  Exactly sum(degree) distinct (user, item) pairs per
    user range; returns (users int32, items int32, ratings f32) on `device`."""
    dev = torch.device(device)
    user_end = n_users if user_end is None else user_end
    g = torch.Generator(device="cpu")
    g.manual_seed(seed * 1000003)
    deg = torch.exp(torch.randn(n_users, generator=g, dtype=torch.float64) + 4.2)
    deg = 20 + deg * max(nnz - 20 * n_users, 0) / deg.sum()
    deg = deg.clamp(max=n_items * 0.5)
    d = torch.floor(deg).long()
    short = nnz - int(d.sum())
    if short > 0:  # distribute the rounding remainder by the fractional parts
        frac = deg - d
        cf = torch.cumsum(frac, 0)
        add = torch.searchsorted(cf / cf[-1], torch.rand(short, generator=g, dtype=torch.float64))
        d += torch.bincount(add.clamp(max=n_users - 1), minlength=n_users)
    del deg
    pop = _zipf_probs(n_items, 0.9, 0.5 * n_users / nnz)
    cdf_i = torch.cumsum(pop, 0)
    cdf_i = (cdf_i / cdf_i[-1]).to(torch.float32).to(dev)
    gi = torch.Generator(device="cpu")
    gi.manual_seed(seed * 15485863)
    perm_items = torch.randperm(n_items, generator=gi).to(dev)
    gv = torch.Generator(device=dev)
    gv.manual_seed(seed * 104729)
    vs = torch.randn((n_items, k_true), generator=gv, device=dev) * 0.35
    out_u, out_i, out_r = [], [], []
    # GLOBAL blocks of consecutive users with about block_ratings ratings each (a
    # block's draws depend only on its global start, so shards reproduce the
    # single-process data); the blocks overlapping [user_begin, user_end) are made
    # whole and filtered to the range
    cum = torch.cumsum(d, 0)
    n_blk = max(1, -(-int(cum[-1]) // block_ratings))
    targets = torch.arange(1, n_blk, dtype=torch.int64) * block_ratings
    bounds = [0] + [int(c) for c in torch.searchsorted(cum, targets, right=True)] + [n_users]
    for b0, b1 in zip(bounds[:-1], bounds[1:]):
        if b1 <= b0 or b1 <= user_begin or b0 >= user_end:
            continue
        ub = b0
        dblk = d[b0:b1].to(dev)
        need = int(dblk.sum())
        gb = torch.Generator(device=dev)
        gb.manual_seed(seed * 7919 + ub)  # per block of GLOBAL users: shard-independent
        users = torch.repeat_interleave(torch.arange(b1 - b0, device=dev), dblk)
        keys = torch.empty(0, dtype=torch.int64, device=dev)
        want = users
        for _ in range(64):
            x = torch.rand(want.numel(), generator=gb, device=dev)
            it = torch.searchsorted(cdf_i, x).clamp(max=n_items - 1)
            keys = torch.unique(torch.cat([keys, want * n_items + it]))
            # per-user counts vs degrees: users still short get more draws
            have = torch.bincount(keys // n_items, minlength=b1 - b0)
            miss = (dblk - have).clamp(min=0)
            if int(miss.sum()) == 0:
                break
            want = torch.repeat_interleave(torch.arange(b1 - b0, device=dev), miss * 2 + 2)
        else:
            raise RuntimeError("synthetic_blocked: could not reach the user degrees")
        # keep exactly deg(u) items per user: random rank within the user
        ku = keys // n_items
        pri = torch.rand(keys.numel(), generator=gb, device=dev)
        order = torch.argsort(ku.double() + pri.double() * 0.5)  # users ascending, random within
        keys = keys[order]
        ku = ku[order]
        start = torch.cumsum(torch.bincount(ku, minlength=b1 - b0), 0) - torch.bincount(
            ku, minlength=b1 - b0)
        rank_in_user = torch.arange(keys.numel(), device=dev) - start[ku]
        keys = keys[rank_in_user < dblk[ku]]
        assert keys.numel() == need
        uu = keys // n_items
        ii = perm_items[keys % n_items]
        us = torch.randn((b1 - b0, k_true), generator=gb, device=dev) * 0.35
        dot = (us[uu] * vs[ii]).sum(1)
        x = 3.6 + dot + 0.8 * torch.randn(need, generator=gb, device=dev)
        r = (torch.round(x * 2) / 2).clamp(0.5, 5.0) if half_stars else torch.round(x).clamp(1.0, 5.0)
        sh = torch.randperm(need, generator=gb, device=dev)  # input order is not sorted
        ug = uu[sh] + ub
        keep = (ug >= user_begin) & (ug < user_end)
        out_u.append(ug[keep].to(torch.int32))
        out_i.append(ii[sh][keep].to(torch.int32))
        out_r.append(r[sh][keep].to(torch.float32))
        del keys, ku, users, uu, ii, us, dot, x, r, sh, order, pri, rank_in_user
    if not out_u:
        z = torch.empty(0, dtype=torch.int32, device=dev)
        return z, z, z.float()
    return torch.cat(out_u), torch.cat(out_i), torch.cat(out_r)


def big_config(name: str = "big1b", device="cuda", rank: int = 0, world: int = 1):
    """configs[3] data for process `rank` of `world` (strong scaling: the user range is
    split in `world` contiguous parts of one global dataset)."""
    n_u, n_i, nnz, half, seed = CONFIGS[name]
    b = n_u * rank // world
    e = n_u * (rank + 1) // world
    return synthetic_blocked(n_u, n_i, nnz, seed=seed, half_stars=half, device=device,
                             user_begin=b, user_end=e)
