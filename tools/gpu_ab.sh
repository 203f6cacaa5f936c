#!/bin/bash
# A/B timing of library variants (tools/ab/variant.py builds) on one workload, the
# variants interleaved twice.  Usage: bash tools/gpu_ab.sh TAG WL STEPS VARIANT... [-- flags]
set -o pipefail
TAG=$1; WL=$2; STEPS=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for rep in 1 2; do
  for v in "$@"; do
    ALS_HIP_DEV=1 ALS_HIP_LIB=$ROOT/tools/ab/libals_$v.so timeout -k 10 400 python -u tools/ab_solve.py $WL $STEPS ${AB_FLAGS:-} >> $OUT/ab_$WL.jsonl 2> $OUT/ab_${WL}_$v.err || { tail -5 $OUT/ab_${WL}_$v.err; exit 1; }
    tail -1 $OUT/ab_$WL.jsonl
  done
done
