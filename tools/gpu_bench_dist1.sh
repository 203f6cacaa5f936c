#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --force-dist --steps 3 --warmup 1 > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err
rc=$?; tail -3 gpurun_out/bench_dist1.err; [ $rc -ne 0 ] && exit $rc
cat gpurun_out/bench_dist1.json | cut -c1-2500
