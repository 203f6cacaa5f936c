#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_big1.json 2> gpurun_out/bench_big1.err
rc=$?; tail -3 gpurun_out/bench_big1.err; [ $rc -ne 0 ] && exit $rc
python3 -c "import json; d=json.load(open('gpurun_out/bench_big1.json')); print(json.dumps({k: d[k] for k in ('value','ms_per_step','configs3','configs4') if k in d})[:3000])"
