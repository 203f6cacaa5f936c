#!/bin/bash
# A/B of library variants (tools/ab/variant.py builds) on a GPU test selection and a
# workload: per variant, the selected tests' reported errors and one ab_solve line.
# Usage: bash tools/gpu_ab_tests.sh TAG 'PYTEST -k EXPR' WL STEPS VARIANT...
set -o pipefail
TAG=$1; K=$2; WL=$3; STEPS=$4; shift 4
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for v in "$@"; do
  LIB=$ROOT/tools/ab/libals_$v.so
  ALS_HIP_DEV=1 ALS_HIP_LIB=$LIB ALS_TEST_REPORT=$OUT/errors_$v.jsonl timeout -k 10 400 \
    python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" \
    > $OUT/tests_$v.log 2>&1 || { tail -5 $OUT/tests_$v.log; exit 1; }
  tail -1 $OUT/tests_$v.log
  ALS_HIP_DEV=1 ALS_HIP_LIB=$LIB timeout -k 10 400 python -u tools/ab_solve.py $WL $STEPS \
    >> $OUT/ab_$WL.jsonl 2> $OUT/ab_${WL}_$v.err || { tail -5 $OUT/ab_${WL}_$v.err; exit 1; }
  tail -1 $OUT/ab_$WL.jsonl
done
