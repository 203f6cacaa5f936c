#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/w1pmc
mkdir -p $OUT
A="$ROOT/tools/ablate.py --w1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python3 $A > $OUT/p1.txt 2>&1 || { tail -3 $OUT/p1.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 $A > $OUT/p2.txt 2>&1 || { tail -3 $OUT/p2.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $OUT/p3 -o run --output-format csv -- python3 $A > $OUT/p3.txt 2>&1 || { tail -3 $OUT/p3.txt; }
python3 $ROOT/tools/pmc_fold.py $OUT/pmc.json $OUT/p1 $OUT/p2 $OUT/p3 | grep ablate
