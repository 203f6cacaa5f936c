#!/bin/bash
# Round-3 closing check on the final tree: smoke() and the full GPU parity suite.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
OUT=gpurun_out/${1:-closing}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
grep "smoke ok" $OUT/smoke.log
ALS_TEST_REPORT=$OUT/errors.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/tests.log | tail -2; exit $rc
