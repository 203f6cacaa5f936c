#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "topk" > gpurun_out/topk_tests.log 2>&1
rc=$?; tail -5 gpurun_out/topk_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/topk_ablate.py --rank 64 --top 10 > gpurun_out/topk_ablate.txt 2>&1 || { tail -5 gpurun_out/topk_ablate.txt; exit 1; }
timeout -k 10 200 python -u tools/topk_ablate.py --rank 128 --top 10 >> gpurun_out/topk_ablate.txt 2>&1 || { tail -5 gpurun_out/topk_ablate.txt; exit 1; }
grep "mode" gpurun_out/topk_ablate.txt
