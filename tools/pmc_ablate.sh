#!/bin/bash
# PMC passes over tools/ablate.py (run on the GPU box).  Usage: bash tools/pmc_ablate.sh TAG
set -o pipefail
TAG=${1:-a1}
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LEVEL_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/p1 -o run --output-format csv -- python3 $ROOT/tools/ablate.py > $OUT/p1.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 $ROOT/tools/ablate.py > $OUT/p2.txt 2>&1 || exit 1
echo done
