#!/bin/bash
# GPU parity suite on the box.  Usage: bash tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-t}; K=${2:-}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
mkdir -p gpurun_out
rm -f gpurun_out/${TAG}_errors.jsonl
ARGS=(tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread)
[ -n "$K" ] && ARGS+=(-k "$K")
ALS_TEST_REPORT=gpurun_out/${TAG}_errors.jsonl timeout -k 10 1000 python -u -m pytest "${ARGS[@]}" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -60
exit $rc
