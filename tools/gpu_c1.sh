#!/bin/bash
# configs[1] (rank 64 explicit) parity subset + bench line (no big objects).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_configs.py -k "configs1 or half_sweep or fit" > gpurun_out/c1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c1_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-big > gpurun_out/c1_bench.json 2> gpurun_out/c1_bench.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/c1_bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/c1_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['topk10_ms'])"
done
