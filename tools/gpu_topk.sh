#!/bin/bash
# K5 (top-k) parity tests and the bench line (top-10 timing, topk_roofline).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "topk" > gpurun_out/topk_tests.log 2>&1
rc=$?; tail -5 gpurun_out/topk_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-big > gpurun_out/topk_bench.json 2> gpurun_out/topk_bench.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/topk_bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/topk_bench.json')); print(d['value'], d['topk10_ms'], json.dumps(d['topk_roofline']))"
