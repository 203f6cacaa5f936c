#!/bin/bash
# W1 explicit Gram A/B: parity suite on the product library, then configs[3] timed with
# the product library and with tools/ab/libals_w1pre1.so (one gather step in flight).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
OUT=gpurun_out/${1:-w1ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit $rc; }
for v in prod pre1 prod; do
  if [ $v = pre1 ]; then L=$PWD/tools/ab/libals_w1pre1.so; else L=; fi
  ALS_HIP_LIB=$L timeout -k 10 300 python bench.py --only c3 --steps 3 --big-steps 3 > $OUT/c3_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/c3_$v.json'))['configs3'];print('$v', round(d['ms_per_iter'],2), {n: round(l['event_ms'],2) for n,l in d['roofline']['launches'].items()})"
done
