#!/usr/bin/env python3
"""ALS hot-path benchmark — BASELINE.json metric
"ratings/sec per ALS iteration (rank 64) at 1/2/4/8 GPUs; top-10 recs/sec".

Primary line (`value`), every N: BASELINE.json configs[1], MovieLens-25M-shaped
synthetic ratings (162,541 users x 59,047 items, 25,000,095 ratings), explicit
ALS, rank 64, regParam 0.1, generated on the device (seeded planted model,
SURVEY.md §8d).  A "step" is one full ALS iteration exactly as Spark runs it:
the item half-sweep (normal equations + Cholesky-equivalent solve for every
item from the user factors) then the user half-sweep, plus the factor
all-gathers when N > 1.  N > 1 is weak scaling of this workload: rank r owns
its own 162,541-user shard of one global dataset (same items); value = all
ratings / max-over-ranks time.

Secondary objects on the same line (BASELINE configs[3] and [4], the
north-star scaling workload; `--no-big` skips them):
  configs3: 1e9-rating power-law synthetic, 10M users x 1M items, rank 128,
            explicit — STRONG scaling: the one global dataset is split over the N
            ranks by user range (each rank generates its range; ShardedALS routes
            ratings to row owners, RCCL all-gathers the factor halves), value =
            1e9 / iteration time.  N = 1 uses the single-GPU engine.
  configs4: recommendForAllUsers top-10 and top-100 on those rank-128 factors,
            over a user sample (262,144 users, split over the ranks; items all
            1M), recs/s = sampled users / time.

Also: `roofline` of the dominant kernel (timed with HIP events on its own
stream; algorithmic bytes and MFMA flops per launch, PMC traffic and
utilisation from the committed rocprofv3 summary), `topk_roofline`,
`cpu_baseline` (the C port of Spark's per-row dspr + dppsv arithmetic,
oracle/als_oracle.c, on the host cores, bounded sample).
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

# MI355X_MICROARCH.md (dense, no sparsity): fp32 matrix/vector 157.3 TF, f16 matrix 2.5 PF
PEAK_FP32_TFLOPS = 157.3
PEAK_F16_MFMA_TFLOPS = 2500.0
PEAK_HBM_GBS = 8000.0
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_summary.json")
BIG_TOPK_SAMPLE = 262144


def dominant_kernel(k: int, implicit: bool) -> str:
    imp = "true" if implicit else "false"
    if k > 64:
        return f"gram_solve_w1_kernel<{imp}>"
    cn = 1 if k <= 16 else (2 if k <= 32 else 4)
    return f"gram_solve_kernel<{cn},{imp}>"


def kp_of(k: int) -> int:
    return 16 if k <= 16 else (32 if k <= 32 else (64 if k <= 64 else 128))


def algorithmic_flops(nnz: int, n_solved: int, k: int) -> float:
    """fp32-grade FLOPs of launch 1 of a half-sweep: symmetric Gram
    k(k+1) and rhs 2k per rating, Cholesky k^3/3 + two triangular solves 2k^2 per row."""
    return nnz * (k * (k + 1) + 2 * k) + n_solved * (k ** 3 / 3 + 2 * k ** 2)


def mfma_issued_flops(nnz: int, n_solved: int, k: int, implicit: bool) -> float:
    """Matrix-core FLOPs the kernel actually issues per launch (what the MFMA pipes do):
    Gram: upper 16x16 tiles x 3 f16 MFMAs (split hi/lo) per 32 ratings (+ 2 rhs MFMAs
    per dims-block, explicit); solve: fp32 16x16x4 trailing / block-row products."""
    cn = kp_of(k) // 16
    nt = cn * (cn + 1) // 2
    per32 = (3 * nt + (0 if implicit else 2 * cn)) * 16 * 16 * 32 * 2
    gram = nnz / 32.0 * per32
    if cn == 8:   # W1: 28 Pm + 84 Schur tile products, 4 x 16x16x4 each
        solve = (28 + 84) * 4 * 16 * 16 * 4 * 2
    else:         # panel LDL^T: trailing tile updates, 4 x 16x16x4 each
        solve = sum((cn - 1 - K) * (cn - K) // 2 for K in range(cn)) * 4 * 16 * 16 * 4 * 2
    return gram + n_solved * solve


def gather_bytes(nnz: int, n_rows: int, k: int) -> float:
    """Algorithmic bytes of launch 1 of a half-sweep: per rating the gathered fp32
    factor row (4k) + column index + rating (8 B); per solved row its output row (4k)
    and row pointer (8 B).  Every byte counted once, no cache reuse assumed."""
    return nnz * (4 * k + 8) + n_rows * (4 * k + 8)


def load_pmc(kernel: str, prefix: bool = False):
    """Per-launch rocprofv3 counters of `kernel` from the committed summary
    (tools/gpu_pmc_r02.sh -> tools/pmc_fold.py), or None.  prefix=True: the first
    kernel whose name starts with `kernel` (template arguments not known here)."""
    try:
        with open(PMC_FILE) as f:
            ks = json.load(f).get("kernels", {})
    except Exception:
        return None
    name = kernel.replace(" ", "")
    if not prefix:
        return ks.get(name)
    hits = sorted(k_ for k_ in ks if k_.startswith(name))
    return ks[hits[0]] if hits else None


def roofline(kernel: str, launch_ms: dict, nnz_rows: list, k: int, implicit: bool):
    """launch_ms: {"item": ms, "user": ms} averages of launch 1 of each half-sweep."""
    launch_s = sum(launch_ms.values()) * 1e-3
    n_launch = len(launch_ms)
    b = sum(gather_bytes(nz, rows, k) for nz, rows in nnz_rows)
    f = sum(algorithmic_flops(nz, rows, k) for nz, rows in nnz_rows)
    fm = sum(mfma_issued_flops(nz, rows, k, implicit) for nz, rows in nnz_rows)
    hbm = b / launch_s / 1e9
    mfma = fm / launch_s / 1e12
    pmc = load_pmc(kernel)
    out = {
        "kernel": kernel,
        "avg_launch_us": 1e6 * launch_s / n_launch,
        "launch_ms": launch_ms,
        "algorithmic_bytes_per_launch": b / n_launch,
        "hbm_view": {"achieved_gbs": hbm, "peak_gbs": PEAK_HBM_GBS, "frac": hbm / PEAK_HBM_GBS},
        "mfma_view": {"issued_flops_per_launch": fm / n_launch, "achieved_tflops": mfma,
                      "peak_tflops": PEAK_F16_MFMA_TFLOPS,
                      "frac": mfma / PEAK_F16_MFMA_TFLOPS,
                      "note": "f16 matrix-core flops issued (split-f16 Gram: 3 MFMAs per "
                              "fp32-grade product) + fp32 16x16x4 solve flops"},
        "fp32_grade_view": {"algorithmic_flops_per_launch": f / n_launch,
                            "achieved_tflops": f / launch_s / 1e12,
                            "peak_tflops": PEAK_FP32_TFLOPS},
    }
    traffic = None
    if pmc:
        t = pmc.get("fetch_bytes_x2", 0.0) + pmc.get("write_bytes", 0.0)
        traffic = t if t > 0 else None
        out["pmc"] = {k_: pmc[k_] for k_ in ("mfma_busy_frac", "valu_busy_frac", "fetch_bytes_x2",
                                             "write_bytes", "pmc_run_avg_ns", "eff_clock_ghz")
                      if k_ in pmc}
        out["pmc"]["source"] = os.path.relpath(PMC_FILE, ROOT)
        if traffic:
            tb = traffic / (1e-6 * out["avg_launch_us"]) / 1e9
            out["pmc_traffic_view"] = {"bytes_per_launch": traffic, "achieved_gbs": tb,
                                       "peak_gbs": PEAK_HBM_GBS, "frac": tb / PEAK_HBM_GBS,
                                       "note": "L2 memory-side bytes (FETCH_SIZE x2 + WRITE_SIZE); "
                                               "below the algorithmic bytes = factor rows "
                                               "re-read from L2 / Infinity Cache"}
        busy = {"valu": pmc.get("valu_busy_frac"), "mfma": pmc.get("mfma_busy_frac"),
                "hbm": (traffic / (1e-6 * out["avg_launch_us"]) / 1e9 / PEAK_HBM_GBS)
                if traffic else None}
        busy = {k_: v for k_, v in busy.items() if v is not None}
        if busy:
            out["limiter"] = max(busy, key=busy.get)
            out["limiter_fracs"] = busy
    # contract: bound in {hbm, mfma}; the larger of the two live fractions
    bound = "hbm" if out["hbm_view"]["frac"] >= out["mfma_view"]["frac"] else "mfma"
    view = out["hbm_view"] if bound == "hbm" else out["mfma_view"]
    out.update({"bound": bound,
                "achieved": view["achieved_gbs"] if bound == "hbm" else view["achieved_tflops"],
                "peak": PEAK_HBM_GBS if bound == "hbm" else PEAK_F16_MFMA_TFLOPS,
                "unit": "GB/s" if bound == "hbm" else "TFLOP/s",
                "frac": view["frac"], "traffic": traffic})
    return out


def topk_roofline(n_q: int, n_v: int, k: int, ms: float, top: int):
    useful = 2.0 * n_q * n_v * k
    kq = max(32, kp_of(k))  # topk_kq (csrc/topk.hip): dims padded to 32/64/128
    issued = 3.0 * 2.0 * n_q * n_v * kq
    s = ms * 1e-3
    out = {"kernel": "topk_split_kernel", "top": top, "n_q": n_q, "n_v": n_v, "rank": k,
           "ms": ms, "recs_per_s": n_q / s,
           "useful_fp32_grade_tflops": useful / s / 1e12,
           "issued_f16_mfma_tflops": issued / s / 1e12,
           "mfma_frac": issued / s / 1e12 / PEAK_F16_MFMA_TFLOPS,
           "bound": "mfma", "unit": "TFLOP/s"}
    # the launched variant (csrc/topk.hip als_topk): <NK, row groups, list kind, 0>
    nk = kq // 32
    if top <= 16:
        rg, tr = 2, (8 if top <= 8 else (12 if top <= 12 else 16))
    elif top <= 128:  # quad register lists, one row group
        rg, tr = 1, (32 if top <= 32 else (64 if top <= 64 else (100 if top <= 100 else 128)))
    else:
        rg, tr = None, 0
    out["kernel"] = f"topk_split_kernel<{nk},{rg if rg else '?'},{tr},0>"
    pmc = load_pmc(out["kernel"]) if rg else None
    if pmc:
        out["pmc"] = {k_: pmc.get(k_) for k_ in ("mfma_busy_frac", "valu_busy_frac",
                                                 "pmc_run_avg_ns")}
        busy = {"valu": pmc.get("valu_busy_frac"), "mfma": pmc.get("mfma_busy_frac")}
        busy = {k_: v for k_, v in busy.items() if v is not None}
        if busy:
            out["limiter"] = max(busy, key=busy.get)
    return out


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


def _timed_topk(Q, n_q, V, n_v, k, top):
    E.topk_rows(Q, n_q, V, n_v, k, top)  # warm (workspace, split table)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    E.topk_rows(Q, n_q, V, n_v, k, top)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def big_single(args, dev):
    """configs[3] (N = 1) and configs[4] on its factors."""
    k = 128
    t0 = time.perf_counter()
    u, i, r = D.big_config("big1b", device=dev)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    core = E.ALSCore(u, i, r, device=dev)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    del u, i, r
    torch.cuda.empty_cache()
    core.init_factors(k, seed=5)
    core.status.zero_()
    steps = max(1, min(args.steps, args.big_steps))
    core.iterate(args.reg)  # warmup
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        core.iterate(args.reg)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    core.check_status()
    res = {"workload": "big1b explicit ALS rank 128 (BASELINE configs[3]), 1 GPU",
           "n_users": core.n_users, "n_items": core.n_items, "nnz": core.nnz, "rank": k,
           "ratings_per_s": core.nnz / dt, "ms_per_iter": 1e3 * dt, "steps": steps,
           "warmup": 1, "datagen_s": t_gen, "build_s": t_build, "scaling": "strong",
           "n_gpus": 1}
    s = min(BIG_TOPK_SAMPLE, core.n_users)
    Q = core.U[:s].contiguous()
    c4 = {"workload": f"recommendForAllUsers on configs[3] factors (BASELINE configs[4]); "
                      f"sample: first {s} users (dense order) x all {core.n_items} items",
          "rank": k}
    for top in (10, 100):
        ms = _timed_topk(Q, s, core.V, core.n_items, k, top)
        c4[f"top{top}_recs_per_s"] = s / (ms * 1e-3)
        c4[f"top{top}_ms"] = ms
        c4[f"top{top}_roofline"] = topk_roofline(s, core.n_items, k, ms, top)
    del core
    torch.cuda.empty_cache()
    return res, c4


def run_single(args):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
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

    # roofline of the dominant kernel (launch 1 of each half-sweep, HIP events on its stream)
    item_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    user_ms = sum(e[2].elapsed_time(e[3]) for e in evs) / args.steps
    roof = roofline(dominant_kernel(k, imp), {"item": item_ms, "user": user_ms},
                    [(ib.nnz, ib.n_light), (ub.nnz, ub.n_light)], k, imp)

    # top-10 recommendations for all users (K5)
    topk_ms = _timed_topk(core.U, core.n_users, core.V, core.n_items, k, 10)
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
        "roofline": roof,
        "topk10_recs_per_s": core.n_users / (topk_ms * 1e-3),
        "topk10_ms": topk_ms,
        "topk_roofline": topk_roofline(core.n_users, core.n_items, k, topk_ms, 10),
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
    del core, ib, ub
    torch.cuda.empty_cache()
    if args.big:
        try:
            out["configs3"], out["configs4"] = big_single(args, dev)
        except Exception as e:  # the primary line must still print
            out["configs3"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    print(json.dumps(out), file=OUT, flush=True)


def _train_triples(core):
    """Recover (user id, item id, rating) of the training set from the user CSR."""
    ub = core.user_block
    deg = ub.row_ptr[1:] - ub.row_ptr[:-1]
    rows = torch.repeat_interleave(torch.arange(ub.n_rows, device=deg.device), deg)
    return core.uidx.ids()[rows], core.iidx.ids()[ub.col.long()], ub.val


def _timed_iterations(sh, reg, warmup, steps, dev):
    for _ in range(warmup):
        sh.iterate(reg)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        sh.iterate(reg)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return float(dt)


def big_distributed(args, dev, rank, world):
    """configs[3] strong scaling over the ranks + configs[4] on the sharded factors."""
    from als_mi355x.distributed import ShardedALS
    k = 128
    t0 = time.perf_counter()
    u, i, r = D.big_config("big1b", device=dev, rank=rank, world=world)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    sh = ShardedALS(u, i, r, device=dev, chunks=args.chunks)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    del u, i, r
    torch.cuda.empty_cache()
    sh.init_factors(k, seed=5)
    steps = max(1, min(args.steps, args.big_steps))
    t = _timed_iterations(sh, args.reg, 1, steps, dev)
    sh.check_status()
    res = {"workload": f"big1b explicit ALS rank 128 (BASELINE configs[3]), {world} GPUs, "
                       "users split by range, RCCL factor all-gather",
           "n_users": sh.n_users, "n_items": sh.n_items, "nnz": sh.nnz, "rank": k,
           "ratings_per_s": sh.nnz / (t / steps), "ms_per_iter": 1e3 * t / steps,
           "steps": steps, "warmup": 1, "datagen_s": t_gen, "build_s": t_build,
           "scaling": "strong", "n_gpus": world, "chunks": sh.users.chunks}
    # configs[4]: each rank scores its share of the user sample against the replicated V
    s_loc = min(BIG_TOPK_SAMPLE // world, sh.users.chunk_rows(rank, 0))
    Vd = sh._dense(False)
    Q = sh.U_loc[0, :s_loc].contiguous()
    c4 = {"workload": f"recommendForAllUsers on configs[3] factors (BASELINE configs[4]); "
                      f"sample: {s_loc} users per rank x {world} ranks x all {sh.n_items} items",
          "rank": k}
    for top in (10, 100):
        E.topk_rows(Q, s_loc, Vd, sh.n_items, k, top)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        E.topk_rows(Q, s_loc, Vd, sh.n_items, k, top)
        torch.cuda.synchronize()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        c4[f"top{top}_recs_per_s"] = s_loc * world / float(dt)
        c4[f"top{top}_ms"] = 1e3 * float(dt)
    return res, c4


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
    t_total = _timed_iterations(sh, args.reg, args.warmup, args.steps, dev)
    out = None
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
    del sh
    torch.cuda.empty_cache()
    if args.big:
        try:
            c3, c4 = big_distributed(args, dev, rank, world)
            if rank == 0:
                out["configs3"], out["configs4"] = c3, c4
        except Exception as e:
            if rank == 0:
                out["configs3"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    if rank == 0:
        print(json.dumps(out), file=OUT, flush=True)
    dist.destroy_process_group()


def _json_stdout():
    """Reserve stdout for the one JSON line: everything else written to fd 1 from here
    on (RCCL prints its version banner there) goes to stderr."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(saved, "w")


OUT = sys.stdout


def main():
    global OUT
    OUT = _json_stdout()
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
    ap.add_argument("--no-big", dest="big", action="store_false",
                    help="skip the configs[3]/[4] (1e9-rating, rank-128) objects")
    ap.add_argument("--big-steps", type=int, default=3,
                    help="timed iterations of configs[3] (at most --steps)")
    ap.add_argument("--chunks", type=int, default=None,
                    help="row chunks per rank for the overlapped all-gathers (N>1)")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the sharded (RCCL) code path even with one rank")
    args = ap.parse_args()
    if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.force_dist:
        run_distributed(args)
    else:
        run_single(args)


if __name__ == "__main__":
    main()
