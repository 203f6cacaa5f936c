#!/bin/bash
# One GPU round-trip: parity tests then a bench line.  Usage: bash gpu_check.sh TAG [bench args]
set -o pipefail
TAG=${1:-run}; shift
mkdir -p gpurun_out
rm -f gpurun_out/${TAG}_errors.jsonl; ALS_TEST_REPORT=gpurun_out/${TAG}_errors.jsonl timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then echo "tests failed rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
cat gpurun_out/${TAG}_bench.json
exit $rc
