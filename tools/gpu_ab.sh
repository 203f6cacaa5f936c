#!/bin/bash
# A/B of two builds of the library (ALS_HIP_LIB) on the configs[1]/configs[2]/explicit-k128
# bench lines, after the full GPU parity suite on the default build.
# Usage: bash tools/gpu_ab.sh TAG ALT_LIB  (ALT_LIB: e.g. the fp32-Schur build, csrc sources
# compiled with -DALS_W1_SCHUR=0 and linked to tools/libals_hip_s0.so)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-ab}; ALT=${2:-tools/libals_hip_s0.so}
mkdir -p gpurun_out
bash tools/gpu_tests.sh ${TAG} > gpurun_out/${TAG}_summary.txt 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_summary.txt; grep FAILED gpurun_out/${TAG}_summary.txt; [ $rc -ne 0 ] && exit $rc
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  ALS_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-big "$@" > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$n.json')); print('$n', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['roofline']['launch_ms'].items()}, round(d['topk10_ms'],3))"
}
DEF=recommender-system-using-apache-spark-mllib-_amd/libals_hip.so
run c2_new $DEF --implicit --rank 128
run c2_old $ALT --implicit --rank 128
run e128_new $DEF --rank 128
run e128_old $ALT --rank 128
run c1_new $DEF
run c1_old $ALT
