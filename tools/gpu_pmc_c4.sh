#!/bin/bash
# PMC passes (same counter sets as gpu_pmc_r02.sh) over the configs[4] top-k run
# (tools/topk_big.py: top-10 and top-100 on configs[3]-shaped factors).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/pmc_c4
mkdir -p $OUT
PA="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES"
PB="GRBM_GUI_ACTIVE FETCH_SIZE"
PC="GRBM_GUI_ACTIVE WRITE_SIZE"
PD="GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVES"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $ROOT/tools/topk_big.py > $OUT/stats.txt 2>&1 || { tail -5 $OUT/stats.txt; exit 1; }
for p in A B C D; do
  eval "cnt=\$P$p"
  timeout -s KILL 150 rocprofv3 --pmc $cnt -d $OUT/$p -o run --output-format csv -- python3 $ROOT/tools/topk_big.py > $OUT/$p.txt 2>&1 || { tail -5 $OUT/$p.txt; exit 1; }
done
grep top $OUT/stats.txt
