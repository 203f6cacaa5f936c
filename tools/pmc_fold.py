"""Fold rocprofv3 outputs into per-workload, per-kernel, per-launch-shape summaries
(profiles/pmc_summary.json, format 2 — what bench.py's rooflines read).

    python tools/pmc_fold.py OUT.json TAG=DIR[,DIR...] [TAG=DIR[,DIR...] ...]

Each TAG is one bench workload (configs1, configs2, configs3, configs4_top10, ...);
its DIRs are the rocprofv3 output directories of that workload's runs: one
`--kernel-trace --stats` run (its *kernel_trace.csv gives per-dispatch durations)
and the separate `--pmc` passes (*counter_collection.csv).  Counters of one
kernel are averaged per dispatch, over all dispatches and separately per grid
size (`by_grid`, keyed by total threads): a half-sweep's item launch and user
launch are the same kernel with different grids.

OUT.json = {"format": 2, "workloads": {TAG: {kernel: {...averages...,
            "by_grid": {grid: {...}}}}}, "sources": {TAG: [dirs]}}

Derived (MI355X_MICROARCH.md "PMC", "HBM" and "DVFS" notes):
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs -> per-XCD busy cycles = /8.
  * SQ_VALU_MFMA_BUSY_CYCLES counts cycles (summed over the SIMDs);
    mfma_busy_frac = MFMA_BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8).
  * SQ_ACTIVE_INST_VALU counts quad-cycles: valu_busy_frac = 4 x it / (1024 x GRBM / 8).
  * SQ_INSTS_VALU_MFMA_MOPS_* count matrix ops in units of 512 FLOP.
  * FETCH_SIZE (KiB) is doubled (gfx950 reports half the bytes of wide reads);
    WRITE_SIZE (KiB) is exact for 16-B stores.
  * trace_avg_ns: kernel-trace average duration (un-profiled run of the same command).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N_SIMD = 1024  # 256 CUs x 4 SIMDs


def short(name):
    name = name.split("(")[0].replace("void ", "").replace("als::", "").replace(" ", "")
    return name[-80:]


def _csvs(dirs, pattern):
    out = []
    for d in dirs:
        out += sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    return out


def derive(ent):
    g = ent.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in ent:
        ent["mfma_busy_frac"] = ent["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * g / 8)
    if g and "SQ_ACTIVE_INST_VALU" in ent:
        ent["valu_busy_frac"] = 4 * ent["SQ_ACTIVE_INST_VALU"] / (N_SIMD * g / 8)
    if g and "SQ_INSTS_VALU" in ent:
        ent["valu_issue_frac"] = 4 * ent["SQ_INSTS_VALU"] / (N_SIMD * g / 8)
    if ent.get("SQ_WAVE_CYCLES", 0) > 0:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in ent:
                ent[c.lower().replace("sq_", "") + "_frac_of_wave"] = ent[c] / ent["SQ_WAVE_CYCLES"]
    if g and "pmc_run_avg_ns" in ent:
        ent["eff_clock_ghz"] = (g / 8) / ent["pmc_run_avg_ns"]
    if "FETCH_SIZE" in ent:
        ent["fetch_bytes_x2"] = 2 * 1024 * ent["FETCH_SIZE"]
    if "WRITE_SIZE" in ent:
        ent["write_bytes"] = 1024 * ent["WRITE_SIZE"]
    for prec in ("F16", "BF16", "F32", "F64", "F8"):
        key = f"SQ_INSTS_VALU_MFMA_MOPS_{prec}"
        if key in ent:
            ent[f"mfma_flop_{prec.lower()}"] = 512 * ent[key]
    return ent


def fold(dirs):
    # counters: (kernel, grid) -> counter -> {dispatch: value}; durations likewise
    per = defaultdict(lambda: defaultdict(dict))
    dur = defaultdict(dict)
    for p in _csvs(dirs, "*counter_collection.csv"):
        with open(p) as f:
            for row in csv.DictReader(f):
                key = (short(row["Kernel_Name"]), int(row["Grid_Size"]))
                did = (p, row["Dispatch_Id"])
                c = per[key][row["Counter_Name"]]
                c[did] = c.get(did, 0.0) + float(row["Counter_Value"])
                try:
                    dur[key][did] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                except (KeyError, ValueError):
                    pass
    trace = defaultdict(list)
    for p in _csvs(dirs, "*kernel_trace.csv"):
        with open(p) as f:
            for row in csv.DictReader(f):
                gs = int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"])
                trace[(short(row["Kernel_Name"]), gs)].append(
                    int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    keys = set(per) | set(trace)
    out = {}
    for kern in sorted({k for k, _ in keys}):
        grids = sorted(g for k, g in keys if k == kern)
        agg_c = defaultdict(list)
        agg_d, agg_t = [], []
        ent = {"by_grid": {}}
        for g in grids:
            e = {}
            cs = per.get((kern, g), {})
            for c, v in cs.items():
                e[c] = sum(v.values()) / len(v)
                agg_c[c] += list(v.values())
            if cs:
                e["dispatches"] = max(len(v) for v in cs.values())
            d = list(dur.get((kern, g), {}).values())
            if d:
                e["pmc_run_avg_ns"] = sum(d) / len(d)
                agg_d += d
            t = trace.get((kern, g), [])
            if t:
                e["trace_avg_ns"] = sum(t) / len(t)
                e["trace_dispatches"] = len(t)
                agg_t += t
            ent["by_grid"][str(g)] = derive(e)
        for c, v in agg_c.items():
            ent[c] = sum(v) / len(v)
        if agg_d:
            ent["pmc_run_avg_ns"] = sum(agg_d) / len(agg_d)
            ent["dispatches"] = len(agg_d)
        if agg_t:
            ent["trace_avg_ns"] = sum(agg_t) / len(agg_t)
            ent["trace_dispatches"] = len(agg_t)
        out[kern] = derive(ent)
    return out


def main():
    dst = sys.argv[1]
    doc = {"format": 2, "workloads": {}, "sources": {}}
    if os.path.exists(dst):  # merge: re-folded workloads replace their old entry
        with open(dst) as f:
            old = json.load(f)
        if old.get("format") == 2:
            doc = old
    for a in sys.argv[2:]:
        tag, dirs = a.split("=", 1)
        dirs = dirs.split(",")
        doc["workloads"][tag] = fold(dirs)
        doc["sources"][tag] = [os.path.basename(d.rstrip("/")) for d in dirs]
    with open(dst, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    for tag in sys.argv[2:]:
        tag = tag.split("=", 1)[0]
        top = sorted(doc["workloads"][tag].items(), key=lambda kv: -kv[1].get("trace_avg_ns", 0))
        for k, v in top[:6]:
            print(tag, k, {c: round(v[c], 4) for c in ("trace_avg_ns", "pmc_run_avg_ns",
                                                       "mfma_busy_frac", "valu_busy_frac",
                                                       "fetch_bytes_x2", "write_bytes") if c in v},
                  "grids", list(v["by_grid"]))


if __name__ == "__main__":
    main()
