#!/bin/bash
# W1 phase ablation + PMC counters of the W1 kernels (explicit k=128 bench).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/w1prof
mkdir -p $OUT
timeout -k 10 200 python3 $ROOT/tools/ablate.py --w1 > $OUT/ablate_w1.txt 2>&1 || { cat $OUT/ablate_w1.txt; exit 1; }
timeout -k 10 200 python3 $ROOT/tools/ablate.py --wg > $OUT/ablate_wg.txt 2>&1 || exit 1
grep -v amdgpu $OUT/ablate_w1.txt $OUT/ablate_wg.txt
B="$ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rmse --rank 128"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python3 $B > $OUT/p1.json 2> $OUT/p1.err || { tail -3 $OUT/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 $B > $OUT/p2.json 2> $OUT/p2.err || { tail -3 $OUT/p2.err; exit 1; }
python3 $ROOT/tools/pmc_fold.py $OUT/pmc.json $OUT/p1 $OUT/p2 | grep -E "w1|wg_kernel|split_table"
