#!/bin/bash
# PMC passes over tools/topk_big.py (configs[4]-shaped top-10 / top-100 on a user
# sample): issue / wait / LDS counters of the top-k kernels, one --pmc pass each.
# Usage (GPU box): bash tools/gpu_pmc_topk.sh TAG [sample]
set -o pipefail
TAG=${1:-tkpmc}; S=${2:-262144}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_LDS"
P2="GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
n=0
for cnt in "$P1" "$P2"; do
  n=$((n + 1))
  timeout -s KILL 400 rocprofv3 --pmc $cnt -d $OUT/p$n -o run --output-format csv -- python3 $ROOT/tools/topk_big.py $S > $OUT/p$n.txt 2>&1 || { tail -5 $OUT/p$n.txt; exit 1; }
  f=$(find $OUT/p$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" > $OUT/p$n.sum <<'EOF'
import collections, csv, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
ids = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if "topk_split_kernel" not in name:
        continue
    key = name.split("(")[0] + " grid " + r.get("Grid_Size", "")
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
    ids[key].add(r.get("Dispatch_Id", ""))
for k, d in acc.items():
    print(k, "dispatches", len(ids[k]))
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:.4g}")
EOF
  cat $OUT/p$n.sum
  rm -rf $OUT/p$n
done
