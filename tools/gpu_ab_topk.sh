#!/bin/bash
# Dev: top-k variants (tools/ab/libals_*.so) vs the product library, alternating.
# Usage: bash tools/gpu_ab_topk.sh TAG v1 v2 ...   (extra args to ab_topk.py via TKARGS)
set -o pipefail
TAG=$1; shift
cd ${GRAFT_REPO_ROOT:-/root/repo}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for v in prod "$@"; do
    if [ $v = prod ]; then L=; else L=$PWD/tools/ab/libals_$v.so; fi
    ALS_HIP_LIB=$L timeout -k 10 400 python tools/ab_topk.py $TKARGS >> $OUT/tk.jsonl 2> $OUT/tk_$v.err || { tail -3 $OUT/tk_$v.err; exit 1; }
    tail -1 $OUT/tk.jsonl
  done
done
