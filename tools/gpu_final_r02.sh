#!/bin/bash
# Round-2 closing evidence: full GPU parity suite, smoke, the default bench line
# (configs[1] + configs[3]/[4] objects), its rocprofv3 kernel-trace stats, and the
# 1-rank sharded (RCCL) path on configs[1].
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-fin}
OUT=gpurun_out/${TAG}
mkdir -p $OUT
bash tools/gpu_tests.sh ${TAG} > $OUT/summary.txt 2>&1
rc=$?; tail -2 $OUT/summary.txt; grep FAILED $OUT/summary.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$OUT/bench_profiled.json 2> $GRAFT_REPO_ROOT/$OUT/prof.err || { tail -5 $GRAFT_REPO_ROOT/$OUT/prof.err; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --force-dist --no-big --no-cpu-baseline > $OUT/bench_dist1.json 2> $OUT/bench_dist1.err || { tail -5 $OUT/bench_dist1.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_dist1.json')); print('dist1', d['value'], d['ms_per_step'])"
