#!/bin/bash
# Round-2 baseline on the GPU box: k=128 phase ablation, configs[2] kernel stats,
# and MFMA/VALU counter passes (each pass its own run, no tracing combined).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/base
mkdir -p $OUT
timeout -k 10 240 python3 $ROOT/tools/ablate.py --wg > $OUT/ablate_wg.txt 2>&1 || { echo "ablate failed"; cat $OUT/ablate_wg.txt; exit 1; }
cat $OUT/ablate_wg.txt
B="$ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --rank 128 --implicit"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/c2trace -o run --output-format csv -- python3 $B > $OUT/c2_bench.json 2> $OUT/c2_trace.err || { echo "trace failed"; tail -5 $OUT/c2_trace.err; exit 1; }
cat $OUT/c2_bench.json
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/c2pmc1 -o run --output-format csv -- python3 $B > $OUT/c2_pmc1.json 2> $OUT/c2_pmc1.err || { echo "pmc1 failed"; tail -5 $OUT/c2_pmc1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 -d $OUT/c2pmc2 -o run --output-format csv -- python3 $B > $OUT/c2_pmc2.json 2> $OUT/c2_pmc2.err || { echo "pmc2 failed"; tail -5 $OUT/c2_pmc2.err; }
echo done
