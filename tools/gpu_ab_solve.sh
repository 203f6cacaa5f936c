#!/bin/bash
# Dev: time solve variants (tools/ab/libals_*.so, built on the CPU host beforehand) and the
# product library on the given workloads, alternating.  Usage: bash tools/gpu_ab_solve.sh TAG "c1 c3" v1 v2 ...
set -o pipefail
TAG=$1; WLS=$2; shift 2
cd ${GRAFT_REPO_ROOT:-/root/repo}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for wl in $WLS; do
  for rep in 1 2; do
    for v in prod "$@"; do
      if [ $v = prod ]; then L=; else L=$PWD/tools/ab/libals_$v.so; fi
      ALS_HIP_LIB=$L timeout -k 10 300 python tools/ab_solve.py $wl 10 >> $OUT/ab.jsonl 2> $OUT/ab_$v.err || { tail -3 $OUT/ab_$v.err; exit 1; }
      tail -1 $OUT/ab.jsonl
    done
  done
done
