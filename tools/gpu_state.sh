#!/bin/bash
# Re-entry check on the box: full GPU parity suite, default bench line, smoke.
# Usage: bash tools/gpu_state.sh TAG
set -o pipefail
TAG=${1:-state}
mkdir -p gpurun_out
bash tools/gpu_tests.sh ${TAG} || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cat gpurun_out/${TAG}_bench.json
