#!/bin/bash
# The driver's default bench line (N = 1, configs[1] + configs[3]/[4] objects + cpu_baseline).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_full.err; exit $rc; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_full.json'))
print(d['value'], d['ms_per_step'], d['topk10_ms'])
print(json.dumps(d.get('configs3'))[:600]); print(json.dumps(d.get('configs4'))[:900]); print(json.dumps(d.get('cpu_baseline'))[:300])"
