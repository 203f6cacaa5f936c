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

Secondary objects on the same line (the other BASELINE configs, each at full size;
`--no-big` skips them):
  configs2: configs[2], the same ML-25M data with implicitPrefs=True, alpha 40,
            rank 128 (YtY Gram + confidence-weighted solves), ms/iter + roofline.
  configs3: configs[3], 1e9-rating power-law synthetic, 10M users x 1M items, rank
            128, explicit — STRONG scaling: the one global dataset is split over the N
            ranks by user range (each rank generates its range; ShardedALS routes
            ratings to row owners, RCCL all-gathers the factor halves), value =
            1e9 / iteration time.  N = 1 uses the single-GPU engine.
  configs4: configs[4], recommendForAllUsers top-10 and top-100 on those rank-128
            factors over ALL 10M users x all 1M items (split over the ranks by user
            range), recs/s = 10M / time.

Every workload carries a roofline of its dominant kernel — ONE kernel: the primal
gram + solve launch of each half-sweep (ALS_PHASE_LAUNCH1), timed alone with HIP
events on the launching stream; the dual-path launch of the short rows
(ALS_PHASE_DUAL) is timed and reported beside it (`dual`).  `frac` = algorithmic
bytes per launch / event time / 8 TB/s; the same over the kernel-trace average of
the PMC profiling runs (`frac_pmc_profile`: tools/gpu_pmc.sh, `bench.py --only W
--steps 3`, a different and shorter run than this one); the PMC traffic / counter DRAM fraction / busy fractions
/ limiter of that workload's own profiled launches (profiles/pmc_summary.json,
keyed by workload, kernel and grid size).  At N = 1 the headline workload's counters
are measured by the run itself: before it touches the GPU, bench.py runs
`bench.py --only c1 --steps 3` under rocprofv3 as five child processes (a kernel
trace and tools/gpu_pmc.sh's four --pmc counter sets) and folds them over the
committed configs1 entry (`live_counters`, `roofline.counters_source`;
`--no-live-pmc` skips it).  `cpu_baseline`: the C port of Spark's
per-row dspr + dppsv arithmetic (oracle/als_oracle.c) on every host core in this
process's affinity set, bounded sample, with the Spark probe (java / pyspark)
recorded.  `--only c1|c2|c3|c4` runs a single workload (profiling passes).
The line records the product library it timed (path + sha256); bench.py refuses
ALS_HIP_LIB (a dev-build override of the library path).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
if os.environ.get("ALS_HIP_LIB"):
    sys.exit("bench.py times the in-tree product library only: unset ALS_HIP_LIB "
             f"(= {os.environ['ALS_HIP_LIB']})")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import _pkgload  # noqa: E402

als = _pkgload.load()
from als_mi355x import datasets as D  # noqa: E402
from als_mi355x import engine as E  # noqa: E402

# MI355X_MICROARCH.md (dense, no sparsity): fp32 matrix/vector 157.3 TF, f16 matrix 2.5 PF
# The arithmetic: fp32 factors and ratings, Gram products on the f16 matrix cores as
# hi.hi + hi.lo + lo.hi of split operands (~2^-21 per product) with fp32 accumulation,
# fp32 block LDL^T solves, fp64 for heavy-row chunk sums, refinement residuals and rescues.
DTYPE = "f32-grade (split-f16 x3 MFMA, fp32 accumulate)"
PEAK_FP32_TFLOPS = 157.3
PEAK_F16_MFMA_TFLOPS = 2500.0
PEAK_HBM_GBS = 8000.0
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_summary.json")
# measured random-row gather rate from an Infinity-Cache-resident table (38 MB, 1,152-B
# rows into LDS; /opt/skills/guides/MI355X_MICROARCH.md "Indexed rows: gather into LDS")
GATHER_IC_GBS = 8600.0
TOPK_WARM_ROWS = 65536


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
    per dims-block, explicit); solve: 16x16 tile products of the block elimination."""
    cn = kp_of(k) // 16
    nt = cn * (cn + 1) // 2
    per32 = (3 * nt + (0 if implicit else 2 * cn)) * 16 * 16 * 32 * 2
    gram = nnz / 32.0 * per32
    if cn == 8:   # W1: 28 Pm + 84 Schur tile products, 4 x 16x16x4 each (fp32-grade)
        solve = (28 + 84) * 4 * 16 * 16 * 4 * 2
    else:         # trailing tile updates, 4 x 16x16x4 each
        solve = sum((cn - 1 - K) * (cn - K) // 2 for K in range(cn)) * 4 * 16 * 16 * 4 * 2
    return gram + n_solved * solve


def gather_bytes(nnz: int, n_rows: int, k: int) -> float:
    """Algorithmic bytes of launch 1 of a half-sweep: per rating the gathered factor row
    (4k) + column index + rating (8 B); per solved row its output row (4k) and row
    pointer (8 B).  Every byte counted once, no cache reuse assumed."""
    return nnz * (4 * k + 8) + n_rows * (4 * k + 8)


# workload -> folded counters measured by this bench run (live_counters), over the file's
_LIVE = {}
# the counter sets of tools/gpu_pmc.sh, one rocprofv3 pass each (within the gfx950
# per-pass block limits: <= 8 SQ_, FETCH_SIZE = 3 TCC_, WRITE_SIZE = 2 TCC_, 1 GRBM_)
LIVE_PASSES = (
    ("T", ["--kernel-trace"]),
    ("A", ["--pmc", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
           "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_VALU_MFMA_BUSY_CYCLES",
           "SQ_INSTS_VALU", "SQ_BUSY_CYCLES"]),
    ("B", ["--pmc", "GRBM_GUI_ACTIVE", "FETCH_SIZE"]),
    ("C", ["--pmc", "GRBM_GUI_ACTIVE", "WRITE_SIZE"]),
    ("D", ["--pmc", "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU_MFMA_MOPS_F16",
           "SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_MFMA",
           "SQ_WAVES"]),
)


def _pmc_doc():
    try:
        with open(PMC_FILE) as f:
            doc = json.load(f)
    except Exception:
        doc = {}
    if _LIVE:
        doc.setdefault("workloads", {}).update(_LIVE)
    return doc


def live_counters(timeout_s: int = 150) -> dict:
    """The headline workload's counters measured by this run: five child processes
    `rocprofv3 <pass> -- python3 bench.py --only c1 --steps 3 --warmup 1` (one kernel-trace
    pass and the four --pmc passes of tools/gpu_pmc.sh), started before this process
    touches the GPU, folded by tools/pmc_fold.py into _LIVE["configs1"] so the primary
    line's roofline.traffic / limiter / busy fractions come from this run, not from the
    committed profiles/pmc_summary.json.  Any failure leaves the committed profile in
    place and is recorded."""
    import importlib.util
    import shutil
    import subprocess
    import tempfile
    rec = {"passes": [p for p, _ in LIVE_PASSES], "workload": "configs1",
           "command": "bench.py --only c1 --steps 3 --warmup 1 --no-rmse"}
    prof = shutil.which("rocprofv3")
    if any(k.startswith("ROCPROF") for k in os.environ):
        # this run is itself profiled (rocprofv3 ... -- python3 bench.py): its children
        # would inherit the profiler's environment; the profile is the counter source
        rec["skipped"] = "run under rocprofv3 (ROCPROF* in the environment)"
        return rec
    if prof is None:
        rec["error"] = "rocprofv3 not on PATH"
        return rec
    t0 = time.perf_counter()
    tmp = tempfile.mkdtemp(prefix="als_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    cmd_tail = ["--", sys.executable, os.path.join(ROOT, "bench.py"), "--only", "c1",
                "--steps", "3", "--warmup", "1", "--no-rmse", "--no-live-pmc"]
    dirs = []
    try:
        for tag, opts in LIVE_PASSES:
            d = os.path.join(tmp, tag)
            with open(d + ".log", "w") as log:
                rc = subprocess.run(["timeout", "-s", "KILL", str(timeout_s), prof] + opts +
                                    ["-d", d, "-o", "run", "--output-format", "csv"] + cmd_tail,
                                    cwd="/tmp", env=env, stdout=log, stderr=subprocess.STDOUT,
                                    ).returncode
            if rc != 0:
                with open(d + ".log") as log:
                    rec["error"] = f"pass {tag} rc {rc}: " + log.read()[-300:]
                return rec
            dirs.append(d)
        spec = importlib.util.spec_from_file_location(
            "pmc_fold", os.path.join(ROOT, "tools", "pmc_fold.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        folded = mod.fold(dirs)
        if not folded.get(dominant_kernel(64, False)):
            rec["error"] = "no counters of the dominant kernel in the passes"
            return rec
        _LIVE["configs1"] = folded
        rec["ok"] = True
        return rec
    except Exception as e:  # the primary line must still print
        rec["error"] = f"{type(e).__name__}: {e}"[:300]
        return rec
    finally:
        rec["seconds"] = time.perf_counter() - t0
        shutil.rmtree(tmp, ignore_errors=True)


def load_pmc(workload: str, kernel: str, grid=None):
    """Per-launch rocprofv3 counters of `kernel` in the committed profile of `workload`
    (tools/gpu_pmc.sh, tools/gpu_pmc_topk.sh -> tools/pmc_fold.py; format 2: workloads -> kernel ->
    all-dispatch averages + by_grid[grid threads]).  grid: the launch's grid size in
    threads, which tells the item launch of a half-sweep from the user launch."""
    ent = _pmc_doc().get("workloads", {}).get(workload, {}).get(kernel.replace(" ", ""))
    if ent is None:
        return None
    if grid is not None:
        return ent.get("by_grid", {}).get(str(int(grid)))
    return ent


def library_record() -> dict:
    """The libals_hip.so this process timed: path and sha256 of its bytes."""
    from als_mi355x import _lib
    path = os.path.realpath(_lib.LIB_PATH)
    with open(path, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    return {"path": os.path.relpath(path, ROOT), "sha256": sha, "abi": _lib.ABI_VERSION}


def _pmc_view(pmc, t_s):
    """Counter view of one launch: traffic, busy fractions, limiter."""
    if not pmc:
        return None
    keep = ("mfma_busy_frac", "valu_busy_frac", "fetch_bytes_x2", "write_bytes", "pmc_run_avg_ns",
            "trace_avg_ns", "eff_clock_ghz", "dispatches", "mfma_flop_f16")
    v = {k_: pmc[k_] for k_ in keep if k_ in pmc}
    traffic = pmc.get("fetch_bytes_x2", 0.0) + pmc.get("write_bytes", 0.0)
    t_run = pmc.get("pmc_run_avg_ns")
    if traffic > 0:
        v["traffic_bytes"] = traffic
        # counters and their own launch time come from the same profiled dispatches
        tt = (t_run * 1e-9) if t_run else t_s
        v["hbm_frac"] = traffic / tt / 1e9 / PEAK_HBM_GBS
    busy = {"valu": pmc.get("valu_busy_frac"), "mfma": pmc.get("mfma_busy_frac"),
            "hbm": v.get("hbm_frac")}
    busy = {k_: x for k_, x in busy.items() if x is not None}
    if busy:
        v["limiter"] = max(busy, key=busy.get)
        v["limiter_fracs"] = busy
    return v


def _combine_pmc(workload: str, parts):
    """Counter view of one launch-1 phase made of several kernels [(kernel, grid)]:
    summed traffic and durations, busy fractions weighted by each kernel's time."""
    ents = [load_pmc(workload, kern, grid) for kern, grid in parts]
    ents = [e for e in ents if e]
    if not ents or len(ents) < len(parts):
        return None
    if len(ents) == 1:
        return ents[0]
    out = {}
    for key in ("fetch_bytes_x2", "write_bytes", "pmc_run_avg_ns", "trace_avg_ns", "mfma_flop_f16"):
        if all(key in e for e in ents):
            out[key] = sum(e[key] for e in ents)
    tw = [e.get("pmc_run_avg_ns", 0.0) for e in ents]
    for key in ("mfma_busy_frac", "valu_busy_frac"):
        if all(key in e for e in ents) and sum(tw) > 0:
            out[key] = sum(e[key] * t for e, t in zip(ents, tw)) / sum(tw)
    return out


def roofline(workload: str, kernel: str, launches: dict, k: int, implicit: bool):
    """Roofline of launch 1 of each half-sweep (the fused Gram + solve kernel; at
    64 < k <= 128 explicit, the n x n dual kernel of the short rows runs in the same
    phase).  launches: {"item"|"user": {"ms": HIP-event average of the phase on the
    launching stream, "nnz": ratings, "rows": rows solved in the phase, "parts":
    [(kernel, grid threads)]}}.  achieved = algorithmic bytes (or modelled issued flops:
    the primal k x k Gram + solve for every row) / event time; frac_pmc_profile uses the
    kernel-trace durations of the same kernels in the PMC profiling runs; traffic / busy
    fractions / limiter / counted MFMA flops come from that workload's PMC passes."""
    out = {"kernel": kernel, "launches": {}}
    tb = tf = tfa = te = tr = 0.0
    traffic = 0.0
    have_traffic = have_trace = True
    busy_w = {}
    for name, L in launches.items():
        b = gather_bytes(L["nnz"], L["rows"], k)
        fm = mfma_issued_flops(L["nnz"], L["rows"], k, implicit)
        fa = algorithmic_flops(L["nnz"], L["rows"], k)
        t = L["ms"] * 1e-3
        ent = {"event_ms": L["ms"], "algorithmic_bytes": b, "hbm_gbs": b / t / 1e9,
               "hbm_frac": b / t / 1e9 / PEAK_HBM_GBS, "mfma_issued_flops": fm,
               "mfma_frac": fm / t / 1e12 / PEAK_F16_MFMA_TFLOPS,
               "fp32_grade_tflops": fa / t / 1e12, "kernels": [list(x) for x in L["parts"]]}
        pv = _pmc_view(_combine_pmc(workload, L["parts"]), t)
        if pv:
            ent["pmc"] = pv
            if pv.get("mfma_flop_f16"):  # counted f16 MFMA flops of the phase's kernels
                ent["mfma_issued_flops_pmc"] = pv["mfma_flop_f16"]
                ent["mfma_frac_pmc"] = pv["mfma_flop_f16"] / t / 1e12 / PEAK_F16_MFMA_TFLOPS
            if pv.get("trace_avg_ns"):
                ent["pmc_profile_trace_ms"] = pv["trace_avg_ns"] * 1e-6
                ent["hbm_frac_pmc_profile"] = b / (pv["trace_avg_ns"] * 1e-9) / 1e9 / PEAK_HBM_GBS
                tr += pv["trace_avg_ns"] * 1e-9
            else:
                have_trace = False
            if "traffic_bytes" in pv:
                traffic += pv["traffic_bytes"]
            else:
                have_traffic = False
            for k_, x in pv.get("limiter_fracs", {}).items():
                busy_w[k_] = busy_w.get(k_, 0.0) + x * t
        else:
            have_trace = have_traffic = False
        out["launches"][name] = ent
        tb += b
        tf += fm
        tfa += fa
        te += t
    n = len(launches)
    hbm = tb / te / 1e9
    mf = tf / te / 1e12
    out.update({
        "avg_launch_us": 1e6 * te / n,
        "algorithmic_bytes_per_launch": tb / n,
        "hbm_view": {"achieved_gbs": hbm, "peak_gbs": PEAK_HBM_GBS, "frac": hbm / PEAK_HBM_GBS},
        # the factor tables of a half-sweep (ML-25M shape: 15-42 MB split tables) sit in
        # the 256 MB Infinity Cache, so the rate the per-rating row gathers can reach is
        # the guide's measured random-row gather rate from such a table, not HBM's
        "gather_view": {"achieved_gbs": hbm, "peak_gbs": GATHER_IC_GBS,
                        "frac": hbm / GATHER_IC_GBS,
                        "note": "vs 8.6 TB/s: random 1,152-B rows gathered into LDS from a 38 MB "
                                "table (Infinity Cache), MI355X_MICROARCH.md 'Indexed rows'; this "
                                "kernel gathers 256-B (k=64) / 512-B (k=128) rows"},
        "mfma_view": {"issued_flops_per_launch": tf / n, "achieved_tflops": mf,
                      "peak_tflops": PEAK_F16_MFMA_TFLOPS, "frac": mf / PEAK_F16_MFMA_TFLOPS,
                      "note": "f16 matrix-core flops issued (split-f16 Gram: 3 MFMAs per "
                              "fp32-grade product) + the solve's tile products"},
        "fp32_grade_view": {"algorithmic_flops_per_launch": tfa / n,
                            "achieved_tflops": tfa / te / 1e12, "peak_tflops": PEAK_FP32_TFLOPS,
                            "note": "Spark's fp32-grade algorithmic flops priced against the fp32 "
                                    "dense MFMA peak, a unit this kernel does not issue (it runs "
                                    "split-f16 MFMA: see mfma_view); not the roofline"},
    })
    # where the counter fields come from: this run's own rocprofv3 child passes
    # (live_counters), else separate passes folded into the committed summary
    out["counters_source"] = (
        "measured by this bench run: rocprofv3 --kernel-trace + 4 --pmc child passes of "
        "`bench.py --only c1 --steps 3 --warmup 1` before the timed run (bench.live_counters)"
        if workload in _LIVE else
        "profiles/pmc_summary.json: rocprofv3 --pmc passes of this workload "
        "(tools/gpu_pmc.sh), not measured in this run")
    busy = {k_: x / te for k_, x in busy_w.items()} if busy_w else {}
    if busy:
        out["limiter"] = max(busy, key=busy.get)
        out["limiter_busy"] = busy[out["limiter"]]
        out["limiter_fracs"] = busy
    if have_traffic and traffic > 0:
        # counter-measured DRAM-side bytes (PMC FETCH_SIZE x 2 + WRITE_SIZE) over the same
        # event time: what actually crossed the memory side (the algorithmic bytes are
        # largely served from the Infinity Cache at the ML-25M shape)
        out["counter_dram_gbs"] = traffic / te / 1e9
        out["counter_dram_frac"] = traffic / te / 1e9 / PEAK_HBM_GBS
    # bound (contract: hbm | mfma) follows the counter limiter of the launches: "hbm"
    # when the DRAM side is the busiest, "mfma" when the issue side is (VALU busy includes
    # the 8 of every 16 cycles an f16 MFMA holds the vector issue port, so a VALU limiter
    # is the compute side too).  Compute-bound: achieved = the f16 matrix-core flops the
    # kernel issues (PMC-counted where profiled, else modelled) / event time against the
    # dense f16 MFMA peak — the unit the kernel runs in; the fp32-grade view (Spark's
    # algorithmic flops vs the fp32 peak) and the algorithmic-bytes view (hbm_view) stay
    # beside it.
    if busy:
        bound = "hbm" if out["limiter"] == "hbm" else "mfma"
    else:
        bound = "hbm" if out["hbm_view"]["frac"] >= out["fp32_grade_view"]["achieved_tflops"] / \
            PEAK_FP32_TFLOPS else "mfma"
    out["fp32_grade_view"]["frac_of_fp32_peak"] = \
        out["fp32_grade_view"]["achieved_tflops"] / PEAK_FP32_TFLOPS
    pmc_f = [L.get("mfma_issued_flops_pmc") for L in out["launches"].values()]
    if all(x for x in pmc_f):
        out["mfma_view"]["issued_flops_per_launch_pmc"] = sum(pmc_f) / n
        out["mfma_view"]["achieved_tflops_pmc"] = sum(pmc_f) / te / 1e12
    if bound == "hbm":
        achieved, peak, unit, frac = hbm, PEAK_HBM_GBS, "GB/s", out["hbm_view"]["frac"]
    else:
        achieved = out["mfma_view"].get("achieved_tflops_pmc", mf)
        peak, unit = PEAK_F16_MFMA_TFLOPS, "TFLOP/s"
        frac = achieved / peak
    out.update({"bound": bound, "achieved": achieved, "peak": peak, "unit": unit, "frac": frac,
                "traffic": traffic / n if (have_traffic and traffic > 0) else None})
    if have_trace and tr > 0:
        issued = sum(pmc_f) if all(x for x in pmc_f) else tf
        out["frac_pmc_profile"] = (tb / tr / 1e9 / PEAK_HBM_GBS) if bound == "hbm" else \
            (issued / tr / 1e12 / PEAK_F16_MFMA_TFLOPS)
        out["pmc_profile_avg_launch_us"] = 1e6 * tr / n
    return out


def topk_variant(k: int, top: int, n_q: int):
    """The kernel als_topk launches (csrc/topk.hip) and its grid in threads:
    (<NK, row groups, list kind>, grid)."""
    nk = max(32, kp_of(k)) // 32
    rg = 2 if n_q >= 4 * 256 * 256 else 1  # two row groups from 4 x 256 x 256 query rows
    if top <= 16:  # register lists (topk_split_rg)
        tr = 8 if top <= 8 else (12 if top <= 12 else 16)
    elif top <= 128:  # key logs, launched in chunks of <= 512 blocks (kTkLogBlocks)
        tr = 32 if top <= 32 else (64 if top <= 64 else (100 if top <= 100 else 128))
    else:
        return f"topk_split_kernel<{nk},?,0>", None
    nw = 8  # wavefronts per workgroup with register lists / key logs (tk_nw)
    blocks = (n_q + 16 * nw * rg - 1) // (16 * nw * rg)
    if top > 16:
        blocks = min(blocks, 512)  # the grid of every launch but the last
    return f"topk_split_kernel<{nk},{rg},{tr}>", blocks * 64 * nw


def topk_roofline(workload: str, n_q: int, n_v: int, k: int, ms: float, top: int):
    """Top-k kernel vs the dense f16 MFMA peak.  Every (query, item) pair gets the hi.hi
    coarse pass (one 16x16x32 f16 MFMA per 32 dims); blocks past the coarse filter add
    hi.lo + lo.hi (two more), so the coarse flops are a floor of what is issued and the
    PMC count (SQ_INSTS_VALU_MFMA_MOPS_F16 x 512) of this workload's launch, where
    profiled, is the total."""
    useful = 2.0 * n_q * n_v * k
    kq = max(32, kp_of(k))  # topk_kq (csrc/topk.hip): dims padded to 32/64/128
    coarse = 2.0 * n_q * n_v * kq
    s = ms * 1e-3
    kern, grid = topk_variant(k, top, n_q)
    out = {"kernel": kern, "top": top, "n_q": n_q, "n_v": n_v, "rank": k,
           "ms": ms, "recs_per_s": n_q / s,
           "useful_fp32_grade_tflops": useful / s / 1e12,
           "coarse_f16_mfma_tflops": coarse / s / 1e12,
           "bound": "mfma", "achieved": coarse / s / 1e12, "peak": PEAK_F16_MFMA_TFLOPS,
           "unit": "TFLOP/s", "frac": coarse / s / 1e12 / PEAK_F16_MFMA_TFLOPS,
           "algorithmic_bytes": 4.0 * (n_q + n_v) * k + 8.0 * n_q * top}
    pv = _pmc_view(load_pmc(workload, kern, grid), s)
    if pv:
        out["pmc"] = pv
        out["traffic"] = pv.get("traffic_bytes")
        issued = pv.get("mfma_flop_f16")
        t_run = pv.get("pmc_run_avg_ns")
        if issued and t_run:
            # counted flops scale with the profiled launch's size (the same n_v, k, top)
            out["issued_f16_mfma_tflops_pmc"] = issued / (t_run * 1e-9) / 1e12
            out["achieved"] = out["issued_f16_mfma_tflops_pmc"]
            out["frac"] = out["achieved"] / PEAK_F16_MFMA_TFLOPS
        if pv.get("trace_avg_ns"):
            out["pmc_profile_trace_ms"] = pv["trace_avg_ns"] * 1e-6
        if "limiter" in pv:
            out["limiter"] = pv["limiter"]
    return out


def _probe_spark():
    """is Spark runnable on this host?  (java on PATH, pyspark importable)"""
    import importlib.util
    import shutil
    java = shutil.which("java")
    try:
        pys = importlib.util.find_spec("pyspark") is not None
    except Exception:
        pys = False
    return {"java": java, "pyspark": pys}


def _cgroup_cpus():
    """CPUs' worth of time the cgroup v2 quota allows (None: no quota)."""
    c = _cgroup_cpu_max()
    try:
        q, per = c.split()
        return None if q == "max" else max(1, -(-int(q) // int(per)))
    except Exception:
        return None


def _cgroup_cpu_max():
    """The cgroup v2 CPU quota of this process ("max 100000" = none), if readable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            return f.read().strip()
    except Exception:
        return None


def cpu_baseline(core: "E.ALSCore", rank: int, reg: float, budget_s: float = 12.0,
                 implicit: bool = False, alpha: float = 1.0):
    """Time the C port (oracle/als_oracle.c, OpenMP) on a bounded prefix of rows of each side;
    extrapolate to ratings/s of a full iteration."""
    import numpy as np
    from oracle import c_oracle
    # every core this process may run on ("N = all host cores"), passed
    # explicitly to the OpenMP port (OMP_NUM_THREADS is left as the host set it) ...
    try:
        affinity = len(os.sched_getaffinity(0))
    except Exception:
        affinity = None
    # ... but a cgroup CPU quota caps the CPU time of the whole process: on the GPU box
    # "1600000 100000" = 16 CPUs' worth over a 256-CPU affinity mask, where 256 threads
    # only time-slice (measured: 8.6e6 ratings/s with 256 threads vs 1.9e7 with 16).
    # threads = the CPUs this process can actually use: min(affinity, quota).
    quota = _cgroup_cpus()
    threads = min(affinity or os.cpu_count(), quota or 1 << 30)
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
    probe = _probe_spark()
    return {"value": core.nnz / total_t, "unit": "ratings/s", "cores": threads, "kind": "port",
            "host_cores": os.cpu_count(), "affinity_cores": affinity, "spark_probe": probe,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "cgroup_cpu_max": _cgroup_cpu_max(), "cgroup_cpus": quota,
            "sample": "oracle/als_oracle.c (Spark dspr+dppsv restated, fp64, OpenMP, "
                      f"{threads} threads) on a row prefix of each side; "
                      + "; ".join(sample_desc)
                      + "; full-iteration time extrapolated as sum over sides of nnz/rate; "
                      + ("Spark not runnable here (java: %s, pyspark importable: %s)"
                         % (probe["java"] or "absent", probe["pyspark"]))}


def _timed_topk(Q, n_q, V, n_v, k, top):
    """recommendForAll over all n_q rows: warmed on a small prefix, then one timed call
    bracketed by HIP events on the launching stream."""
    E.topk_rows(Q, min(n_q, TOPK_WARM_ROWS), V, n_v, k, top)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    idx, sc = E.topk_rows(Q, n_q, V, n_v, k, top)
    e1.record()
    torch.cuda.synchronize()
    del idx, sc
    return e0.elapsed_time(e1)


def _half_sweep_timed(core, block, Y, X, k, reg, imp, alpha, yty, ev=None):
    """solve_half in its phases (the normal call's order), the primal launch and the
    dual launch each bracketed by events on the launching stream (ev = 3 events)."""
    P = E  # phase bits: engine.PHASE_*
    E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws,
                 P.PHASE_PREP | P.PHASE_RSCALE)
    if ev is not None:
        ev[0].record()
    E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws, P.PHASE_LAUNCH1)
    if ev is not None:
        ev[1].record()
    E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws, P.PHASE_DUAL)
    if ev is not None:
        ev[2].record()
    E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws,
                 P.PHASE_LAUNCH2 | P.PHASE_RESCUE)


def _iteration(core, k, reg, imp, alpha, evs=None):
    """One ALS iteration in Spark's order (ALS.train loop): items from users, then users
    from items; implicit: YtY of the source side before each half-sweep (computeYtY)."""
    yty = E.compute_yty(core.U, core.n_users, k, core.ws_yty) if imp else None
    _half_sweep_timed(core, core.item_block, core.U, core.V, k, reg, imp, alpha, yty,
                      evs[0:3] if evs else None)
    yty = E.compute_yty(core.V, core.n_items, k, core.ws_yty) if imp else None
    _half_sweep_timed(core, core.user_block, core.V, core.U, k, reg, imp, alpha, yty,
                      evs[3:6] if evs else None)


def _n_dual(block, k: int, imp: bool, reg: float = 0.1) -> int:
    return 0 if (imp or reg <= 0) else block.n_dual(k)


def dual_kernel(k: int) -> str:
    return f"gram_solve_dual_kernel<{128 if k > 64 else 64}>"


def _launch1_parts(block, k: int, imp: bool, reg: float = 0.1):
    """Kernels als_solve_half launches for a half-sweep's light rows: [(kernel, grid
    threads)] — the primal launch (ALS_PHASE_LAUNCH1: chunk tasks + primal light rows),
    then, when there are dual rows, the dual launch (ALS_PHASE_DUAL)."""
    kern = dominant_kernel(k, imp)
    n_dual = _n_dual(block, k, imp, reg)
    parts = [(kern, 64 * (block.n_chunks + block.n_light - n_dual))]
    if n_dual > 0:
        parts.append((dual_kernel(k), 64 * n_dual))
    return parts


def dual_view(workload: str, k: int, blocks: dict, ms: dict, reg: float):
    """The dual launch of each half-sweep (explicit short rows): event time, algorithmic
    bytes (each rating's factor row + index + rating, each row's output) and HBM
    fraction, plus that kernel's PMC view when profiled."""
    out = {"kernel": dual_kernel(k), "launches": {}}
    for name, blk in blocks.items():
        nd = _n_dual(blk, k, False, reg)
        if nd == 0:
            continue
        b = gather_bytes(blk.dual_nnz(k), nd, k)
        t = ms[name] * 1e-3
        ent = {"rows": nd, "nnz": blk.dual_nnz(k), "event_ms": ms[name], "algorithmic_bytes": b,
               "hbm_frac": b / t / 1e9 / PEAK_HBM_GBS}
        pv = _pmc_view(load_pmc(workload, dual_kernel(k), 64 * nd), t)
        if pv:
            ent["pmc"] = pv
        out["launches"][name] = ent
    return out if out["launches"] else None


def rescued_rows(core, k, reg, imp, alpha):
    """One more (untimed) iteration, reading the rescue list's length before each
    RESCUE phase: rows the fp32-grade path handed to the fp64 re-solve (split window,
    pivot spread, failed pivot) per half-sweep — 0 on well-scaled data."""
    out = {}
    for name, block, Y, X, n_src in (("item", core.item_block, core.U, core.V, core.n_users),
                                     ("user", core.user_block, core.V, core.U, core.n_items)):
        yty = E.compute_yty(Y, n_src, k, core.ws_yty) if imp else None
        E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws,
                     E.PHASE_ALL & ~E.PHASE_RESCUE)
        torch.cuda.synchronize()
        out[name] = int(core.ws.buf[8:12].view(torch.int32).item())  # scale word 2
        E.solve_half(block, Y, X, k, reg, imp, alpha, yty, core.status, core.ws,
                     E.PHASE_RESCUE)
    torch.cuda.synchronize()
    return out


def timed_fit(core, workload, k, reg, imp, alpha, steps, warmup):
    """warmup + `steps` timed iterations from the seeded start; per-iteration wall time
    and the event times of the primal and dual launches of each half-sweep
    -> (ms_per_iter, roofline of the primal kernel, dual view)."""
    core.init_factors(k, seed=5)
    core.schedule_for(imp)  # the engine's heavy-row task length for this fit
    core.status.zero_()
    for _ in range(warmup):
        _iteration(core, k, reg, imp, alpha)
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(steps)]
    t0 = time.perf_counter()
    for s in range(steps):
        _iteration(core, k, reg, imp, alpha, evs[s])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    core.check_status()
    ib, ub = core.item_block, core.user_block

    def avg(a, b):
        return sum(e[a].elapsed_time(e[b]) for e in evs) / steps
    launches = {}
    for name, blk, o in (("item", ib, 0), ("user", ub, 3)):
        nd = _n_dual(blk, k, imp, reg)
        launches[name] = {"ms": avg(o, o + 1), "nnz": blk.nnz - (blk.dual_nnz(k) if nd else 0),
                          "rows": blk.n_light - nd, "parts": _launch1_parts(blk, k, imp, reg)[:1]}
    roof = roofline(workload, dominant_kernel(k, imp), launches, k, imp)
    dual = None if imp else dual_view(workload, k, {"item": ib, "user": ub},
                                      {"item": avg(1, 2), "user": avg(4, 5)}, reg)
    roof["fp64_rescued_rows_per_half_sweep"] = rescued_rows(core, k, reg, imp, alpha)
    return 1e3 * dt, roof, dual


def configs2(core, args):
    """BASELINE configs[2]: the ML-25M shape, implicitPrefs=True alpha=40, rank 128."""
    k, alpha = 128, 40.0
    ms, roof, _ = timed_fit(core, "configs2", k, args.reg, True, alpha, args.steps, args.warmup)
    return {"workload": "ml25m implicit alpha=40 ALS rank 128 (BASELINE configs[2]), 1 GPU",
            "n_users": core.n_users, "n_items": core.n_items, "nnz": core.nnz, "rank": k,
            "alpha": alpha, "ratings_per_s": core.nnz / (ms * 1e-3), "ms_per_iter": ms,
            "steps": args.steps, "warmup": args.warmup, "roofline": roof}


def big_single(args, dev, want_c3=True, want_c4=True):
    """configs[3] (N = 1) and configs[4] on its factors (all 10M users)."""
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
    steps = max(1, min(args.steps, args.big_steps))
    c3 = c4 = None
    if want_c3:
        ms, roof, dual = timed_fit(core, "configs3", k, args.reg, False, 1.0, steps, 1)
        c3 = {"workload": "big1b explicit ALS rank 128 (BASELINE configs[3]), 1 GPU",
              "n_users": core.n_users, "n_items": core.n_items, "nnz": core.nnz, "rank": k,
              "ratings_per_s": core.nnz / (ms * 1e-3), "ms_per_iter": ms, "steps": steps,
              "warmup": 1, "datagen_s": t_gen, "build_s": t_build, "scaling": "strong",
              "n_gpus": 1, "roofline": roof, "dual": dual,
              "schedule": {"item": [core.item_block.n_light, core.item_block.n_heavy,
                                    core.item_block.n_chunks],
                           "user": [core.user_block.n_light, core.user_block.n_heavy,
                                    core.user_block.n_chunks]}}
    else:  # the factor state the full run reaches: seed + 1 warmup + `steps` iterations
        core.init_factors(k, seed=5)
        for _ in range(1 + steps):
            core.iterate(args.reg)
        torch.cuda.synchronize()
    if want_c4:
        c4 = {"workload": f"recommendForAllUsers on the configs[3] factors (BASELINE "
                          f"configs[4]): all {core.n_users} users x all {core.n_items} items",
              "rank": k, "n_users": core.n_users, "n_items": core.n_items}
        for top in (10, 100):
            ms = _timed_topk(core.U, core.n_users, core.V, core.n_items, k, top)
            c4[f"top{top}_recs_per_s"] = core.n_users / (ms * 1e-3)
            c4[f"top{top}_ms"] = ms
            c4[f"top{top}_roofline"] = topk_roofline("configs4", core.n_users, core.n_items, k,
                                                     ms, top)
    del core
    torch.cuda.empty_cache()
    return c3, c4


def run_single(args, live=None):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if args.only in ("c3", "c4"):
        c3, c4 = big_single(args, dev, args.only == "c3", args.only == "c4")
        print(json.dumps({"configs3": c3} if c3 else {"configs4": c4}), file=OUT, flush=True)
        return
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
    if args.only == "c2":
        print(json.dumps({"configs2": configs2(core, args)}), file=OUT, flush=True)
        return
    k = args.rank
    imp, alpha = args.implicit, args.alpha
    wl = "configs2" if (imp and k == 128) else "configs1"
    ms_per_step, roof, dual = timed_fit(core, wl, k, args.reg, imp, alpha, args.steps,
                                        args.warmup)
    value = core.nnz / (ms_per_step * 1e-3)
    ib, ub = core.item_block, core.user_block
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
        "dtype": DTYPE,
        "data": "synthetic (seeded planted low-rank model on device; ML-25M shape)",
        "config": {"workload": f"{args.config} {mode} ALS rank {k} (BASELINE configs[{cfg_idx}])",
                   "n_users": core.n_users, "n_items": core.n_items, "nnz": core.nnz,
                   "rank": k, "regParam": args.reg, "implicitPrefs": imp, "alpha": alpha,
                   "parallelism": "dp1"},
        "roofline": roof,
        "live_counters": live,
        "dual": dual,
        "library": library_record(),
        "topk10_recs_per_s": core.n_users / (topk_ms * 1e-3),
        "topk10_ms": topk_ms,
        "topk_roofline": topk_roofline("configs1", core.n_users, core.n_items, k, topk_ms, 10),
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
    if args.big and not imp and args.config == "ml25m":
        try:
            out["configs2"] = configs2(core, args)
        except Exception as e:  # the primary line must still print
            out["configs2"] = {"error": f"{type(e).__name__}: {e}"[:300]}
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
    sh = ShardedALS(u, i, r, device=dev, chunks=args.chunks, **_sharded_opts(args))
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
           "scaling": "strong", "n_gpus": world, "chunks": sh.users.chunks,
           "exchange": dict(sh.exchange_stats(k), mode=sh.exchange, pipelined=sh.pipeline)}
    # configs[4]: each rank scores its own users (every chunk of its range) against the
    # replicated V; time = max over ranks
    Vd = sh._dense(False)
    cs = sh.users.cstarts[rank]
    c4 = {"workload": f"recommendForAllUsers on the configs[3] factors (BASELINE configs[4]): "
                      f"all {sh.n_users} users (each rank its own range) x all {sh.n_items} "
                      "items", "rank": k}
    for top in (10, 100):
        E.topk_rows(sh.U_loc[0], min(sh.users.chunk_rows(rank, 0), TOPK_WARM_ROWS), Vd,
                    sh.n_items, k, top)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for c in range(sh.users.chunks):
            n_c = int(cs[c + 1] - cs[c])
            if n_c > 0:
                idx, sc = E.topk_rows(sh.U_loc[c], n_c, Vd, sh.n_items, k, top)
                del idx, sc
        torch.cuda.synchronize()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        c4[f"top{top}_recs_per_s"] = sh.n_users / float(dt)
        c4[f"top{top}_ms"] = 1e3 * float(dt)
    return res, c4


def _sharded_opts(args) -> dict:
    """--exchange / --pipeline -> ShardedALS arguments (defaults: RCCL ring all-gather,
    no pipelined item half-sweep)."""
    pipe = {"off": None, "on": True, "auto": "auto"}[args.pipeline]
    return {"exchange": args.exchange, "pipeline": pipe}


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
    sh = ShardedALS(u, i, r, device=dev, chunks=args.chunks, **_sharded_opts(args))
    del u, i, r
    k = args.rank
    sh.init_factors(k, seed=5)
    t_total = _timed_iterations(sh, args.reg, args.warmup, args.steps, dev)
    ex = dict(sh.exchange_stats(k), mode=sh.exchange, pipelined=sh.pipeline)
    out = None
    if rank == 0:
        out = {
            "metric": "ratings/sec per ALS iteration (rank 64)",
            "exchange": ex,
            "value": sh.nnz / (t_total / args.steps),
            "unit": "ratings/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * t_total / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": DTYPE,
            "data": "synthetic (seeded planted model; one ML-25M-shaped user shard per rank)",
            "config": {"workload": f"{args.config} x{world} users explicit ALS rank {k} "
                                   "(weak scaling of BASELINE configs[1])",
                       "n_users": sh.users.n, "n_items": sh.items.n, "nnz": sh.nnz,
                       "rank": k, "regParam": args.reg, "parallelism": f"dp{world}"},
            "roofline": None,
            "cpu_baseline": None,
            "library": library_record(),
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
    ap.add_argument("--exchange", choices=("ring", "peers"), default="ring",
                    help="N > 1: factor exchange (RCCL ring all-gather or batched P2P to all peers)")
    ap.add_argument("--pipeline", choices=("off", "on", "auto"), default="off",
                    help="N > 1: the pipelined item half-sweep (auto: the exchange model)")
    ap.add_argument("--only", choices=("c1", "c2", "c3", "c4"), default=None,
                    help="profiling runs: only this workload (c4 fits c3 untimed first)")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the sharded (RCCL) code path even with one rank")
    ap.add_argument("--no-live-pmc", dest="live_pmc", action="store_false",
                    help="N = 1: skip the rocprofv3 child passes that measure the headline "
                         "kernel's counters in this run (the committed profile is used)")
    args = ap.parse_args()
    if args.only == "c1":
        args.big, args.cpu_baseline = False, False
    if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.force_dist:
        run_distributed(args)
    else:
        # before this process touches the GPU: the child passes get the card to themselves
        live = live_counters() if (args.live_pmc and args.only is None and args.rank == 64
                                   and not args.implicit and args.config == "ml25m") else None
        run_single(args, live)


if __name__ == "__main__":
    main()
