#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/topk_ablate.py --rank 64 --top 10 > gpurun_out/topk_ablate.txt 2>&1 || { tail -5 gpurun_out/topk_ablate.txt; exit 1; }
timeout -k 10 200 python -u tools/topk_ablate.py --rank 128 --top 10 >> gpurun_out/topk_ablate.txt 2>&1 || { tail -5 gpurun_out/topk_ablate.txt; exit 1; }
grep "mode" gpurun_out/topk_ablate.txt
