"""Fold rocprofv3 --pmc counter_collection.csv files into per-kernel, per-launch
averages (one entry per short kernel name), plus derived utilisation figures.

    python tools/pmc_fold.py OUT.json DIR_OR_CSV [DIR_OR_CSV ...]
    python tools/pmc_fold.py OUT.json TAG=DIR[,DIR...] [TAG=DIR[,DIR...] ...]

The second form folds each group (one workload's passes) separately and merges
them; a kernel name present in several groups keeps the FIRST group's entry
(e.g. topk_split_kernel of the rank-64 run).  OUT.json = {"kernels": {...},
"groups": {kernel: tag}, "sources": {tag: [dirs]}}.

Derived (MI355X_MICROARCH.md "PMC" and "DVFS" notes):
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs -> per-XCD busy cycles = /8.
  * SQ_VALU_MFMA_BUSY_CYCLES counts cycles (summed over the SIMDs);
    mfma_busy_frac = MFMA_BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8).
  * SQ_INSTS_VALU_MFMA_MOPS_* count matrix ops in units of 512 FLOP.
  * FETCH_SIZE (KiB) is doubled for 16-B/lane reads (gfx950 correction);
    WRITE_SIZE (KiB) is exact for 16-B stores.
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


def files(args):
    out = []
    for a in args:
        if os.path.isdir(a):
            out += sorted(glob.glob(os.path.join(a, "**", "*counter_collection.csv"), recursive=True))
        else:
            out.append(a)
    return out


def fold(paths):
    # (kernel, counter) -> list of per-dispatch values
    per = defaultdict(lambda: defaultdict(dict))
    dur = defaultdict(dict)
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                did = (p, row["Dispatch_Id"])
                per[k][row["Counter_Name"]][did] = (per[k][row["Counter_Name"]].get(did, 0.0)
                                                    + float(row["Counter_Value"]))
                try:
                    dur[k][did] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                except (KeyError, ValueError):
                    pass
    out = {}
    for k, cs in per.items():
        ent = {"dispatches": max(len(v) for v in cs.values())}
        for c, v in cs.items():
            ent[c] = sum(v.values()) / len(v)
        if dur[k]:
            ent["pmc_run_avg_ns"] = sum(dur[k].values()) / len(dur[k])
        g = ent.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in ent:
            ent["mfma_busy_frac"] = ent["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * g / 8)
        if g and "SQ_ACTIVE_INST_VALU" in ent:  # quad-cycles per wave
            ent["valu_busy_frac"] = 4 * ent["SQ_ACTIVE_INST_VALU"] / (N_SIMD * g / 8)
        if g and "SQ_INSTS_VALU" in ent:  # 4 issue cycles per wave64 instruction
            ent["valu_issue_frac"] = 4 * ent["SQ_INSTS_VALU"] / (N_SIMD * g / 8)
        if "SQ_WAVE_CYCLES" in ent and ent["SQ_WAVE_CYCLES"] > 0:
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
        out[k] = ent
    return out


def main():
    dst = sys.argv[1]
    args = sys.argv[2:]
    if args and all("=" in a for a in args):
        res, groups, sources = {}, {}, {}
        for a in args:
            tag, dirs = a.split("=", 1)
            dirs = dirs.split(",")
            sources[tag] = [os.path.basename(d.rstrip("/")) for d in dirs]
            for k, v in fold(files(dirs)).items():
                if k not in res:
                    res[k], groups[k] = v, tag
        doc = {"kernels": res, "groups": groups, "sources": sources}
    else:
        res = fold(files(args))
        doc = {"kernels": res}
    with open(dst, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1].get("pmc_run_avg_ns", 0))[:12]:
        print(k, {c: (round(x, 4) if isinstance(x, float) else x) for c, x in v.items()})


if __name__ == "__main__":
    main()
