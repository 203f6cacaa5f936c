#!/bin/bash
# GPU step for top-k work: the top-k parity tests, then the A/B timing of
# tools/ab/libtk_{base,new}.so on configs[4]-shaped factors.
# Usage: bash tools/gpu_topk_ab.sh TAG [sample_users] [pytest -k expr]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-tk}; S=${2:-262144}; K=${3:-topk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -60
[ $rc -ne 0 ] && { grep -E "^E |Error" $OUT/tests.log | head -40; exit $rc; }
timeout -k 10 400 python -u tools/ab/topk_ab.py $S > $OUT/ab.log 2>&1
rc=$?
cat $OUT/ab.log | grep -v Warning | tail -20
exit $rc
