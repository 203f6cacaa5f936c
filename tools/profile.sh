#!/bin/bash
# rocprofv3 evidence for bench.py (run ON the GPU box via gpurun):
#   1. kernel trace + stats of a short bench run      -> gpurun_out/prof_<tag>/trace
#   2. PMC pass FETCH_SIZE (own run, no tracing)      -> gpurun_out/prof_<tag>/pmc_fetch
#   3. PMC pass WRITE_SIZE (own run)                   -> gpurun_out/prof_<tag>/pmc_write
# then tools/pmc_summary.py folds them into profiles/<tag>_*.{csv,json}.
# Usage: bash tools/profile.sh r01 [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
cd /tmp && export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="$ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace pass failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 $BENCH > $OUT/fetch_bench.json 2> $OUT/fetch.err || { echo "fetch pass failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 $BENCH > $OUT/write_bench.json 2> $OUT/write.err || { echo "write pass failed"; exit 1; }
python3 $ROOT/tools/pmc_summary.py $OUT $TAG
