#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
bash tools/gpu_tests.sh w1 "128 or 100 or 65 or 72 or configs2 or mixed" || exit 1
timeout -k 10 200 python3 tools/ablate.py --w1 > gpurun_out/ablate_w1.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/ablate_w1.txt
for f in c2:--implicit e128: ; do tag=${f%%:*}; arg=${f#*:}
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --rank 128 $arg > gpurun_out/w1_bench_$tag.json 2> gpurun_out/w1_bench_$tag.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/w1_bench_$tag.json')); print('$tag', d['ms_per_step'], d['roofline']['launch_ms'])"
done
