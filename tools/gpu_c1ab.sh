#!/bin/bash
# configs[1] A/B: the product library vs tools/ab/libals_w1pre1.so, alternating.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
OUT=gpurun_out/${1:-c1ab}
mkdir -p $OUT
if [ "${2:-}" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit $rc; }
fi
for v in prod alt prod alt; do
  if [ $v = alt ]; then L=$PWD/tools/ab/libals_w1pre1.so; else L=; fi
  ALS_HIP_LIB=$L timeout -k 10 200 python bench.py --only c1 --steps 20 --warmup 5 > $OUT/c1_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$OUT/c1_$v.json'));print('$v', round(d['ms_per_step'],4), {n: round(l['event_ms'],4) for n,l in d['roofline']['launches'].items()}, 'topk10', round(d['topk10_ms'],3))"
done
