#!/usr/bin/env python3
"""ALS hot-path benchmark — BASELINE.json metric "ratings/sec per ALS iteration (rank 64)".

Workload (BASELINE.json configs[1]): MovieLens-25M-shaped synthetic ratings,
162,541 users x 59,047 items, 25,000,095 ratings, explicit ALS, rank 64,
regParam 0.1 — generated on the device (seeded planted model).
A "step" is one full ALS iteration exactly as Spark runs it: the item
half-sweep (normal equations + Cholesky for every item from the user factors)
then the user half-sweep, plus the factor all-gathers when N > 1.

N > 1 (launched by torch.distributed.run, one rank per GPU): weak scaling —
every rank generates its own 162,541-user shard of one global dataset (same
59,047 items), ratings are routed once to their user-row and item-row owners
(all_to_all), and each half-sweep ends with an RCCL all_gather of the updated
factor half.  value = total ratings of all ranks / max-over-ranks time.

Also reported: `roofline` of the dominant kernel (gram_solve_kernel<4,false>,
timed with HIP events on its own stream), `cpu_baseline` (the C port of
Spark's per-row dspr + dppsv arithmetic, oracle/als_oracle.c, on the host
cores, bounded sample), top-10 recs/s (recommendForAllUsers(10), N = 1 only)
and the training RMSE.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _pkgload  # noqa: E402

als = _pkgload.load()
from als_mi355x import datasets as D  # noqa: E402
from als_mi355x import engine as E  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix, spec
PEAK_HBM_GBS = 8000.0


def dominant_kernel(k: int, implicit: bool) -> str:
    imp = "true" if implicit else "false"
    if k > 64:
        return f"gram_solve_wg_kernel<{imp}>"
    cn = 1 if k <= 16 else (2 if k <= 32 else 4)
    return f"gram_solve_kernel<{cn},{imp}>"


def gram_flops(nnz: int, n_solved: int, k: int) -> float:
    """Algorithmic FLOPs of launch 1 of a half-sweep: symmetric Gram k(k+1)/2 FMAs and the
    rhs k FMAs per rating, plus Cholesky (k^3/3) + two triangular solves (2k^2) per row
    solved in the same launch."""
    return nnz * (k * (k + 1) + 2 * k) + n_solved * (k ** 3 / 3 + 2 * k ** 2)


def gather_bytes(nnz: int, n_rows: int, k: int) -> float:
    """Algorithmic bytes of launch 1 of a half-sweep: per rating the gathered fp32
    factor row (4k) + column index + rating (8 B); per solved row its output row (4k)
    and row pointer (8 B).  Every byte counted once, no cache reuse assumed."""
    return nnz * (4 * k + 8) + n_rows * (4 * k + 8)


def load_pmc(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (tools/profile.sh -> tools/pmc_summary.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
        ent = d.get(kernel.replace(" ", ""))
        return None if ent is None else ent.get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(core: "E.ALSCore", rank: int, reg: float, budget_s: float = 12.0,
                 implicit: bool = False, alpha: float = 1.0):
    """Time the C port (oracle/als_oracle.c, OpenMP) on a bounded prefix of rows of each side;
    extrapolate to ratings/s of a full iteration."""
    import numpy as np
    from oracle import c_oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    U = core.U[:, :rank].contiguous().cpu().numpy()
    V = core.V[:, :rank].contiguous().cpu().numpy()
    total_t = 0.0
    sample_desc = []
    for name, block, Y in (("item", core.item_block, U), ("user", core.user_block, V)):
        ptr = block.row_ptr.cpu().numpy()
        col = block.col.cpu().numpy()
        val = block.val.cpu().numpy()
        # calibrate on a small prefix, then size the sample to ~budget/2 seconds
        rate = None
        target = 200_000
        for _ in range(2):
            nrow = int(np.searchsorted(ptr, min(target, ptr[-1]), side="right"))
            nrow = max(1, min(nrow, len(ptr) - 1))
            sub_ptr = ptr[:nrow + 1].copy()
            nz = int(sub_ptr[-1])
            t0 = time.perf_counter()
            c_oracle.half_sweep(sub_ptr, col[:nz], val[:nz], Y, reg, implicit=implicit,
                                alpha=alpha, threads=threads)
            dt = time.perf_counter() - t0
            rate = nz / dt
            target = int(rate * budget_s / 2)
        total_t += block.nnz / rate
        sample_desc.append(f"{name} side: first {nrow} rows ({nz} ratings) in {dt:.2f}s")
    return {"value": core.nnz / total_t, "unit": "ratings/s", "cores": threads, "kind": "port",
            "sample": "oracle/als_oracle.c (Spark dspr+dppsv restated, fp64, OpenMP) on a row "
                      "prefix of each side; " + "; ".join(sample_desc)
                      + "; full-iteration time extrapolated as sum over sides of nnz/rate"}


def run_single(args):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n_u, n_i, nnz_cfg, _, _ = D.CONFIGS[args.config]
    t0 = time.perf_counter()
    u, i, r = D.synthetic_config(args.config, device=dev)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    core = E.ALSCore(u, i, r, device=dev)
    ev1.record()
    torch.cuda.synchronize()
    build_ms = ev0.elapsed_time(ev1)
    del u, i, r
    k = args.rank
    core.init_factors(k, seed=5)
    core.status.zero_()
    ib, ub = core.item_block, core.user_block

    imp, alpha = args.implicit, args.alpha

    def iteration(evs=None):
        # Spark order: items from users, then users from items (ALS.train loop);
        # implicit: YtY of the source side before each half-sweep (computeYtY)
        yty = E.compute_yty(core.U, core.n_users, k, core.ws) if imp else None
        E.solve_half(ib, core.U, core.V, k, args.reg, imp, alpha, yty, core.status, core.ws, 12)
        if evs is not None:
            evs[0].record()
        E.solve_half(ib, core.U, core.V, k, args.reg, imp, alpha, yty, core.status, core.ws, 1)
        if evs is not None:
            evs[1].record()
        E.solve_half(ib, core.U, core.V, k, args.reg, imp, alpha, yty, core.status, core.ws, 2)
        yty = E.compute_yty(core.V, core.n_items, k, core.ws) if imp else None
        E.solve_half(ub, core.V, core.U, k, args.reg, imp, alpha, yty, core.status, core.ws, 12)
        if evs is not None:
            evs[2].record()
        E.solve_half(ub, core.V, core.U, k, args.reg, imp, alpha, yty, core.status, core.ws, 1)
        if evs is not None:
            evs[3].record()
        E.solve_half(ub, core.V, core.U, k, args.reg, imp, alpha, yty, core.status, core.ws, 2)

    for _ in range(args.warmup):
        iteration()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    t_start = time.perf_counter()
    for s in range(args.steps):
        iteration(evs[s])
    torch.cuda.synchronize()
    t_total = time.perf_counter() - t_start
    core.check_status()
    ms_per_step = 1000.0 * t_total / args.steps
    value = core.nnz / (t_total / args.steps)

    # roofline of the dominant kernel (launch 1 of each half-sweep)
    item_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    user_ms = sum(e[2].elapsed_time(e[3]) for e in evs) / args.steps
    f_item = gram_flops(ib.nnz, ib.n_light, k)
    f_user = gram_flops(ub.nnz, ub.n_light, k)
    b_item = gather_bytes(ib.nnz, ib.n_light, k)
    b_user = gather_bytes(ub.nnz, ub.n_light, k)
    launch_s = (item_ms + user_ms) * 1e-3
    achieved = (b_item + b_user) / launch_s / 1e9
    tflops = (f_item + f_user) / launch_s / 1e12
    avg_launch_us = 1000.0 * (item_ms + user_ms) / 2
    dominant = dominant_kernel(k, imp)
    traffic = load_pmc(dominant)

    # top-10 recommendations for all users (K5), timed with events after one warm run
    core.recommend_users(10)
    torch.cuda.synchronize()
    t0e, t1e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0e.record()
    core.recommend_users(10)
    t1e.record()
    torch.cuda.synchronize()
    topk_ms = t0e.elapsed_time(t1e)
    mode = f"implicit alpha={alpha:g}" if imp else "explicit"
    cfg_idx = 2 if (imp and k == 128) else 1
    out = {
        "metric": "ratings/sec per ALS iteration (rank 64)" if k == 64 and not imp
                  else f"ratings/sec per ALS iteration (rank {k}, {mode})",
        "value": value,
        "unit": "ratings/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded planted low-rank model on device; ML-25M shape)",
        "config": {"workload": f"{args.config} {mode} ALS rank {k} (BASELINE configs[{cfg_idx}])",
                   "n_users": core.n_users, "n_items": core.n_items, "nnz": core.nnz,
                   "rank": k, "regParam": args.reg, "implicitPrefs": imp, "alpha": alpha,
                   "parallelism": "dp1"},
        "roofline": {"bound": "hbm", "kernel": dominant,
                     "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                     "avg_launch_us": avg_launch_us,
                     "algorithmic_bytes_per_launch": (b_item + b_user) / 2,
                     "launch_ms": {"item": item_ms, "user": user_ms},
                     "flops_view": {"algorithmic_flops_per_launch": (f_item + f_user) / 2,
                                    "achieved_tflops": tflops,
                                    "note": "fp32-grade Gram on f16 MFMA (3 products per "
                                            "fp32 product, k<=64); peak f16 dense 2500 TF, "
                                            "fp32 157.3 TF"}},
        "topk10_recs_per_s": core.n_users / (topk_ms * 1e-3),
        "topk10_ms": topk_ms,
        "csr_build_ms": build_ms,
        "datagen_s": t_gen,
        "schedule": {"item": [ib.n_light, ib.n_heavy, ib.n_chunks],
                     "user": [ub.n_light, ub.n_heavy, ub.n_chunks]},
    }
    if args.rmse:
        rmse, n = core.rmse(*_train_triples(core))
        out["train_rmse"] = rmse
    if args.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(core, k, args.reg, args.cpu_budget, imp, alpha)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)


def _train_triples(core):
    """Recover (user id, item id, rating) of the training set from the user CSR."""
    ub = core.user_block
    deg = ub.row_ptr[1:] - ub.row_ptr[:-1]
    rows = torch.repeat_interleave(torch.arange(ub.n_rows, device=deg.device), deg)
    return core.uidx.uniq[rows], core.iidx.uniq[ub.col.long()], ub.val


def run_distributed(args):
    from als_mi355x.distributed import ShardedALS
    for k_, v_ in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29517"), ("RANK", "0"),
                   ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
        os.environ.setdefault(k_, v_)
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    rank, world = dist.get_rank(), dist.get_world_size()
    u, i, r = D.synthetic_config(args.config, device=dev, shard=rank)
    sh = ShardedALS(u, i, r, device=dev, chunks=args.chunks)
    del u, i, r
    k = args.rank
    sh.init_factors(k, seed=5)
    for _ in range(args.warmup):
        sh.iterate(args.reg)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sh.iterate(args.reg)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    t_total = float(dt)
    if rank == 0:
        out = {
            "metric": "ratings/sec per ALS iteration (rank 64)",
            "value": sh.nnz / (t_total / args.steps),
            "unit": "ratings/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * t_total / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded planted model; one ML-25M-shaped user shard per rank)",
            "config": {"workload": f"{args.config} x{world} users explicit ALS rank {k} "
                                   "(weak scaling of BASELINE configs[1])",
                       "n_users": sh.users.n, "n_items": sh.items.n, "nnz": sh.nnz,
                       "rank": k, "regParam": args.reg, "parallelism": f"dp{world}"},
            "roofline": None,
            "cpu_baseline": None,
        }
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="ml25m", choices=sorted(D.CONFIGS))
    ap.add_argument("--rank", type=int, default=64)
    ap.add_argument("--reg", type=float, default=0.1)
    ap.add_argument("--implicit", action="store_true", help="implicitPrefs=True (configs[2])")
    ap.add_argument("--alpha", type=float, default=40.0)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-rmse", dest="rmse", action="store_false")
    ap.add_argument("--chunks", type=int, default=None,
                    help="row chunks per rank for the overlapped all-gathers (default 4 at N>1)")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the sharded (RCCL) code path even with one rank")
    args = ap.parse_args()
    if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.force_dist:
        run_distributed(args)
    else:
        run_single(args)


if __name__ == "__main__":
    main()
