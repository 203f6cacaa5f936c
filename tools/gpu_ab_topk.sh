#!/bin/bash
# A/B timing of top-k library variants (tools/ab/variant.py builds) on the configs[4]
# sample (tools/topk_big.py), interleaved twice; every variant's results are compared
# with the first one's.  Usage: bash tools/gpu_ab_topk.sh TAG SAMPLE VARIANT...
set -o pipefail
TAG=$1; S=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
FIRST=$1
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = "$FIRST" ]; then X="TOPK_SAVE=$OUT/ref.pt"; else X="TOPK_CMP=$OUT/ref.pt"; fi
    env $X ALS_HIP_DEV=1 ALS_HIP_LIB=$ROOT/tools/ab/libals_$v.so timeout -k 10 300 python -u tools/topk_big.py $S >> $OUT/ab_topk.txt 2> $OUT/ab_topk_$v.err || { tail -5 $OUT/ab_topk_$v.err; exit 1; }
    grep "libals_$v.so" $OUT/ab_topk.txt | tail -4
  done
done
rm -f $OUT/ref.pt
