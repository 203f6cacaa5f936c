#!/bin/bash
# Round-3 GPU step: parity suite (optionally -k filtered), then optionally the bench.
# Usage: bash tools/gpu_r03.sh TAG [pytest -k expr] [bench args...]
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r3}; K=${2:-}; shift 2; BARGS=("$@")
OUT=gpurun_out/${TAG}
mkdir -p $OUT
ARGS=(tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread)
[ -n "$K" ] && [ "$K" != "none" ] && ARGS+=(-k "$K")
if [ "$K" != "none" ]; then
  ALS_TEST_REPORT=$OUT/errors.jsonl timeout -k 10 900 python -u -m pytest "${ARGS[@]}" > $OUT/tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/tests.log | tail -40
  [ $rc -ne 0 ] && { tail -40 $OUT/tests.log; exit $rc; }
fi
if [ ${#BARGS[@]} -gt 0 ] && [ "${BARGS[0]}" != "nobench" ]; then
  timeout -k 10 600 python bench.py "${BARGS[@]}" > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value', d.get('value'), 'ms', d.get('ms_per_step'))
for k in ('configs2','configs3','configs4'):
    if k in d: print(k, json.dumps(d[k])[:600])
"
fi
