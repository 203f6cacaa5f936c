#!/bin/bash
# Profiles of the bench workloads, one `bench.py --only W` run per pass:
# a --kernel-trace --stats run and four --pmc passes (counter sets below, each
# within the gfx950 per-pass limits), folded per workload into
# gpurun_out/pmc_run/pmc_summary.json (tools/pmc_fold.py, format 2).
# Usage: bash tools/gpu_pmc_run.sh c1 c2 c3 c4     (any subset)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/pmc_run
mkdir -p $OUT
[ -f $ROOT/profiles/pmc_summary.json ] && [ ! -f $OUT/pmc_summary.json ] && cp $ROOT/profiles/pmc_summary.json $OUT/pmc_summary.json
PA="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES"
PB="GRBM_GUI_ACTIVE FETCH_SIZE"
PC="GRBM_GUI_ACTIVE WRITE_SIZE"
PD="GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVES"
declare -A TAG=([c1]=configs1 [c2]=configs2 [c3]=configs3 [c4]=configs4)
for w in "$@"; do
  B="$ROOT/bench.py --only $w --steps 3 --warmup 1 --big-steps 3 --no-rmse"
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/T_$w -o run --output-format csv -- python3 $B > $OUT/bench_$w.json 2> $OUT/T_$w.err || { tail -5 $OUT/T_$w.err; exit 1; }
  dirs=$OUT/T_$w
  for p in A B C D; do
    eval "cnt=\$P$p"
    timeout -s KILL 300 rocprofv3 --pmc $cnt -d $OUT/${p}_$w -o run --output-format csv -- python3 $B > $OUT/${p}_$w.txt 2>&1 || { tail -5 $OUT/${p}_$w.txt; exit 1; }
    dirs=$dirs,$OUT/${p}_$w
  done
  python3 $ROOT/tools/pmc_fold.py $OUT/pmc_summary.json ${TAG[$w]}=$dirs > $OUT/fold_$w.txt 2>&1 || { cat $OUT/fold_$w.txt; exit 1; }
  grep -E "gram_solve|topk_split|dual" $OUT/fold_$w.txt | cut -c1-400
  # keep only the folded summary + stats csv (the raw per-dispatch csvs are large)
  cp $OUT/T_$w/run_kernel_stats.csv $OUT/kernel_stats_$w.csv 2>/dev/null || cp $(find $OUT/T_$w -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats_$w.csv
  rm -rf $OUT/T_$w $OUT/A_$w $OUT/B_$w $OUT/C_$w $OUT/D_$w
done
