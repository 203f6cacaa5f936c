#!/bin/bash
# Phase ablation of the explicit light-row kernels (tools/ablate.py) + one PMC pass.
# Usage: bash tools/gpu_ablate.sh TAG
set -o pipefail
TAG=${1:-abl}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python -u tools/ablate.py --rank 64 > $OUT/abl64.txt 2>&1 || { tail -5 $OUT/abl64.txt; exit 1; }
cat $OUT/abl64.txt
timeout -k 10 300 python -u tools/ablate.py --rank 128 > $OUT/abl128.txt 2>&1 || { tail -5 $OUT/abl128.txt; exit 1; }
cat $OUT/abl128.txt
cd /tmp && export TMPDIR=/tmp
PA="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $PA -d $OUT/P -o run --output-format csv -- python3 $ROOT/tools/ablate.py --rank 64 > $OUT/pmc.txt 2>&1 || { tail -5 $OUT/pmc.txt; exit 1; }
f=$(find $OUT/P -name "*counter_collection.csv" | head -1)
python3 - "$f" > $OUT/pmc_summary.txt <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for row in csv.DictReader(open(sys.argv[1])):
    kn = row["Kernel_Name"][:60]
    agg[kn][row["Counter_Name"]] += float(row["Counter_Value"])
    if row["Counter_Name"] == "GRBM_GUI_ACTIVE":
        n[kn] += 1
for kn, c in agg.items():
    busy = c.get("SQ_BUSY_CYCLES", 1) or 1
    wc = c.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{kn:60s} n={n[kn]:3d} valu/busy={c['SQ_ACTIVE_INST_VALU']/busy:.3f} mfma/busy={c['SQ_VALU_MFMA_BUSY_CYCLES']/busy:.3f} "
          f"insts_valu={c['SQ_INSTS_VALU']/max(n[kn],1):.3g} insts_mfma={c['SQ_INSTS_MFMA']/max(n[kn],1):.3g} "
          f"any/wave={c['SQ_ACTIVE_INST_ANY']/wc:.3f} wait/wave={c['SQ_WAIT_INST_ANY']/wc:.3f}")
PY
cat $OUT/pmc_summary.txt
rm -rf $OUT/P
