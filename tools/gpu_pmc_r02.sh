#!/bin/bash
# Round-2 profiles of the bench workloads: kernel-trace stats + PMC passes for
#   c1 = configs[1] (rank 64 explicit, the primary line) and
#   c2 = configs[2] (rank 128 implicit alpha 40).
# Output: gpurun_out/pmc_r02/{stats,A,B,C,D}_{c1,c2}, folded into pmc_summary.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/pmc_r02
mkdir -p $OUT
B="$ROOT/bench.py --steps 5 --warmup 2 --no-big --no-cpu-baseline --no-rmse"
declare -A ARGS=([c1]="" [c2]="--implicit --rank 128")
PA="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES"
PB="GRBM_GUI_ACTIVE FETCH_SIZE"
PC="GRBM_GUI_ACTIVE WRITE_SIZE"
PD="GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVES"
for c in c1 c2; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $OUT/stats_$c -o run --output-format csv -- python3 $B ${ARGS[$c]} > $OUT/bench_$c.json 2> $OUT/stats_$c.err || { tail -5 $OUT/stats_$c.err; exit 1; }
  for p in A B C D; do
    eval "cnt=\$P$p"
    timeout -s KILL 150 rocprofv3 --pmc $cnt -d $OUT/${p}_$c -o run --output-format csv -- python3 $B ${ARGS[$c]} > $OUT/${p}_$c.txt 2>&1 || { tail -5 $OUT/${p}_$c.txt; exit 1; }
  done
done
python3 $ROOT/tools/pmc_fold.py $OUT/pmc_summary.json \
  c1=$OUT/A_c1,$OUT/B_c1,$OUT/C_c1,$OUT/D_c1 c2=$OUT/A_c2,$OUT/B_c2,$OUT/C_c2,$OUT/D_c2 > $OUT/fold.txt
grep -E "gram_solve|topk|reduce_solve" $OUT/fold.txt | cut -c1-600
