#!/bin/bash
# configs[2] (rank 128 implicit) parity subset + bench line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_configs.py -k "128 or implicit or yty or configs2 or heavy or mixed" > gpurun_out/c2_tests.log 2>&1
rc=$?; tail -4 gpurun_out/c2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --implicit --rank 128 --steps 5 --warmup 2 --no-cpu-baseline --no-big > gpurun_out/c2_bench.json 2> gpurun_out/c2_bench.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/c2_bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/c2_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['topk10_ms'])"
