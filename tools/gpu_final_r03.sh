#!/bin/bash
# Round-3 closing measurement: the driver's default bench line, then the same command
# under rocprofv3 --kernel-trace --stats (its kernel summary backs the line's rooflines).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/${1:-final}
mkdir -p $OUT
cd $ROOT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'topk10', d['topk10_ms'])
print('c2', d['configs2']['ms_per_iter'], 'c3', d['configs3']['ms_per_iter'], 'c4', d['configs4']['top10_ms'], d['configs4']['top100_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/T -o run --output-format csv -- python3 $ROOT/bench.py > $OUT/bench_traced.json 2> $OUT/traced.err || { tail -5 $OUT/traced.err; exit 1; }
cp $(find $OUT/T -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
rm -rf $OUT/T
head -12 $OUT/kernel_stats.csv | cut -c1-200
