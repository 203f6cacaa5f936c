#!/bin/bash
# W1 (one wave per k=128 system) check: parity tests, then A/B bench vs the round-1 wg path.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
bash tools/gpu_tests.sh w1 "128 or 100 or 65 or 72 or configs2 or mixed" || exit 1
for path in w1 wg; do
  ALS_K128_PATH=$path timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --rank 128 --implicit > gpurun_out/w1_bench_c2_$path.json 2> gpurun_out/w1_bench_c2_$path.err || exit 1
  ALS_K128_PATH=$path timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --rank 128 > gpurun_out/w1_bench_e128_$path.json 2> gpurun_out/w1_bench_e128_$path.err || exit 1
done
for f in gpurun_out/w1_bench_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['ms_per_step'], d['roofline']['launch_ms'], d['topk10_ms'])"; done
