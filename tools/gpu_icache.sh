#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/icache
mkdir -p $OUT
A="$ROOT/tools/ablate.py --w1"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python3 $A > $OUT/p1.txt 2>&1 || { tail -5 $OUT/p1.txt; exit 1; }
python3 $ROOT/tools/pmc_fold.py $OUT/pmc.json $OUT/p1 | grep ablate
