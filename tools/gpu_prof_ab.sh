#!/bin/bash
# Dev: per-kernel rocprofv3 stats of tools/ab_solve.py on one workload for the product
# library and tools/ab/libals_<v>.so variants.  Usage: bash tools/gpu_prof_ab.sh TAG WL v1 v2 ...
# -> gpurun_out/TAG/<v>.stats.csv (the trace itself stays on the box).
set -o pipefail
TAG=$1; WL=$2; shift 2
cd ${GRAFT_REPO_ROOT:-/root/repo}
R=$PWD; OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in prod "$@"; do
  if [ $v = prod ]; then L=; else L=$R/tools/ab/libals_$v.so; fi
  rm -rf /tmp/prof_$v
  ALS_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$v -o run --output-format csv -- python3 tools/ab_solve.py $WL 3 > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  S=$(find /tmp/prof_$v -name "*kernel_stats.csv" | head -1)
  cp "$S" $OUT/$v.stats.csv
  grep '^{' $OUT/$v.log | tail -1
done
