#!/bin/bash
# Counter passes of the top-k kernels on a configs[4] sample (tools/ab/topk_once.py):
# one --kernel-trace --stats run + PMC passes, each within the gfx950 per-pass limits.
# Usage: bash tools/gpu_topk_pmc.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$1
mkdir -p $OUT
B="$ROOT/tools/ab/topk_once.py 262144"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/T -o run --output-format csv -- python3 $B > $OUT/T.txt 2>&1 || { tail -5 $OUT/T.txt; exit 1; }
PA="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES"
PB="GRBM_GUI_ACTIVE FETCH_SIZE"
PD="GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
dirs=$OUT/T
for p in A B D; do
  eval "cnt=\$P$p"
  timeout -s KILL 200 rocprofv3 --pmc $cnt -d $OUT/$p -o run --output-format csv -- python3 $B > $OUT/$p.txt 2>&1 || { tail -5 $OUT/$p.txt; exit 1; }
  dirs=$dirs,$OUT/$p
done
python3 $ROOT/tools/pmc_fold.py $OUT/pmc.json topk=$dirs > $OUT/fold.txt 2>&1 || { cat $OUT/fold.txt; exit 1; }
grep -E "topk_split" $OUT/fold.txt | cut -c1-600
cp $(find $OUT/T -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
rm -rf $OUT/T $OUT/A $OUT/B $OUT/D
