#!/bin/bash
# Round-4 GPU pass: the parity suite, the driver's bench command, and the same command
# under rocprofv3 --kernel-trace --stats (its summary backs the headline roofline).
# Usage: bash tools/gpu_r04.sh TAG [tests|bench|prof ...]   (default: all three)
set -o pipefail
TAG=${1:-r04}; shift
STEPS=${@:-tests bench prof}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
echo "nproc $(nproc) affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" | tee $OUT/host.txt
for s in $STEPS; do
  case $s in
    tests)
      ALS_TEST_REPORT=$OUT/errors.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
      rc=$?; grep -E "FAILED|ERROR" $OUT/tests.log | head -20; tail -1 $OUT/tests.log
      [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
      python3 tools/bench_summary.py $OUT/bench.json ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/T -o run --output-format csv -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_traced.json 2> $OUT/traced.err ) || { tail -5 $OUT/traced.err; exit 1; }
      cp $(find $OUT/T -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
      rm -rf $OUT/T
      python3 tools/bench_summary.py $OUT/bench_traced.json $OUT/kernel_stats.csv ;;
  esac
done
