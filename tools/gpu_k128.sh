#!/bin/bash
# rank-128 (W1) parity subset + configs[2] bench + explicit rank-128 bench.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_checkpoint.py -k "128 or implicit or yty or configs2 or heavy or mixed or resume or failed" > gpurun_out/k128_tests.log 2>&1
rc=$?; tail -3 gpurun_out/k128_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --implicit --rank 128 --steps 5 --warmup 2 --no-cpu-baseline --no-big > gpurun_out/k128_imp.json 2> gpurun_out/k128_imp.err || { tail -5 gpurun_out/k128_imp.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/k128_imp.json')); print('implicit', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
timeout -k 10 300 python -u bench.py --rank 128 --steps 5 --warmup 2 --no-cpu-baseline --no-big > gpurun_out/k128_exp.json 2> gpurun_out/k128_exp.err || { tail -5 gpurun_out/k128_exp.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/k128_exp.json')); print('explicit', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
