#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ablate.py --w1 > gpurun_out/w1lat.txt 2>&1 || { tail -5 gpurun_out/w1lat.txt; exit 1; }
timeout -k 10 300 python -u tools/ablate.py --w1 --local-cols >> gpurun_out/w1lat.txt 2>&1 || { tail -5 gpurun_out/w1lat.txt; exit 1; }
grep "mode" gpurun_out/w1lat.txt
