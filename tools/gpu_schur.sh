#!/bin/bash
# Dev: W1 phase times with the Schur/Pm products as fp32 MFMA (s0) or split f16 (s1),
# then the k>32 parity subset and the configs[1]/configs[2] bench lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for v in 0 1; do
  echo "== variant s$v"
  ALS_DEV_SO=tools/libals_dev_s$v.so timeout -k 10 200 python -u tools/ablate.py --w1 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/gpu_tests.sh sch "128 or 100 or 65 or 72 or 48 or 64 or configs or mixed or fit or failed" > gpurun_out/sch_summary.txt 2>&1
rc=$?; tail -3 gpurun_out/sch_summary.txt; grep -c PASSED gpurun_out/sch_summary.txt; grep FAILED gpurun_out/sch_summary.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --implicit --rank 128 --steps 5 --warmup 2 --no-cpu-baseline --no-big > gpurun_out/sch_c2.json 2> gpurun_out/sch_c2.err || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-big > gpurun_out/sch_c1.json 2> gpurun_out/sch_c1.err || exit 1
for f in sch_c2 sch_c1; do python3 -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['topk10_ms'])"; done
