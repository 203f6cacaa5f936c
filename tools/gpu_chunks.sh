#!/bin/bash
# Chunked all-gather overlap on the 1-rank RCCL path: C = 1, 2, 4 (configs[1]).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for C in 1 2 4; do
  timeout -k 10 300 python -u bench.py --force-dist --no-big --chunks $C --steps 10 --warmup 3 > gpurun_out/chunks_$C.json 2> gpurun_out/chunks_$C.err || { tail -5 gpurun_out/chunks_$C.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/chunks_$C.json')); print('C=$C', d['ms_per_step'], d['value'])"
done
