#!/bin/bash
# One GPU pass on the box (gpurun).  Usage:
#   bash tools/gpu.sh TAG STEP [STEP ...]
# STEP: tests            the GPU parity suite (errors -> $OUT/errors.jsonl)
#       tests:EXPR       the suite filtered by pytest -k EXPR
#       bench            the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#       bench:ARGS       bench.py with ARGS (comma-separated, e.g. bench:--only,c3)
#       prof             the driver's command under rocprofv3 --kernel-trace --stats
#       smoke            __graft_entry__.smoke()
# Every step has its own time limit; the first failing step ends the pass.
set -o pipefail
TAG=${1:-run}; shift
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
echo "nproc $(nproc) affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" > $OUT/host.txt
n=0
for s in "$@"; do
  n=$((n + 1))
  case $s in
    tests|tests:*)
      K=${s#tests}; K=${K#:}
      ARGS=(tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread)
      [ -n "$K" ] && ARGS+=(-k "$K")
      ALS_TEST_REPORT=$OUT/errors.jsonl timeout -k 10 900 python -u -m pytest "${ARGS[@]}" > $OUT/tests$n.log 2>&1
      rc=$?; grep -E "FAILED|ERROR" $OUT/tests$n.log | head -20; tail -1 $OUT/tests$n.log
      [ $rc -eq 0 ] || exit $rc ;;
    bench|bench:*)
      A=${s#bench}; A=${A#:}; A=${A//,/ }
      [ -z "$A" ] && A="--gpus 1 --steps 20 --warmup 5"
      timeout -k 10 900 python -u bench.py $A > $OUT/bench$n.json 2> $OUT/bench$n.err || { tail -5 $OUT/bench$n.err; exit 1; }
      python3 tools/bench_summary.py $OUT/bench$n.json ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/T -o run --output-format csv -- python3 $ROOT/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_traced.json 2> $OUT/traced.err ) || { tail -5 $OUT/traced.err; exit 1; }
      cp $(find $OUT/T -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
      rm -rf $OUT/T
      python3 tools/bench_summary.py $OUT/bench_traced.json $OUT/kernel_stats.csv ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
      tail -3 $OUT/smoke.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
