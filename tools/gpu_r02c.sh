#!/bin/bash
# Full GPU parity suite, then configs[4] top-k timing and the default bench line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r02c}
mkdir -p gpurun_out
bash tools/gpu_tests.sh ${TAG} > gpurun_out/${TAG}_summary.txt 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_summary.txt; grep FAILED gpurun_out/${TAG}_summary.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/topk_big.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['topk10_ms'], d['configs3']['ms_per_iter'], d['configs4']['top10_ms'], d['configs4']['top100_ms'])"
