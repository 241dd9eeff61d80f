#!/bin/bash
# A/B/C… of library variants, alternated on one box: the in-tree library (A) and tools/variants/<tag>.so.
# usage: bash tools/r6/abn.sh <out-dir> <reps> "<tag1> <tag2> ..." <bench args...>
set -u
OUT=$1; REPS=$2; TAGS=$3; shift 3
mkdir -p "$OUT"
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp "$LIB" "$OUT/.libA.so"
rc=0
for rep in $(seq 1 $REPS); do
  for v in A $TAGS; do
    if [ $v = A ]; then cp "$OUT/.libA.so" "$LIB"; else cp "tools/variants/$v.so" "$LIB"; fi
    YFM_BENCH_DUMP="$OUT/$v$rep.npy" timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-host-rate > "$OUT/$v$rep.json" 2> "$OUT/$v$rep.err" || { rc=$?; break 2; }
    python -c "import json; d=json.load(open('$OUT/$v$rep.json')); print('$v$rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
cp "$OUT/.libA.so" "$LIB"
rm -f "$OUT/.libA.so"
[ $rc = 0 ] && for v in $TAGS; do python -c "
import numpy as np
a, b = np.load('$OUT/A1.npy'), np.load('$OUT/${v}1.npy')
f = np.isfinite(a) & np.isfinite(b)
same = np.array_equal(a, b, equal_nan=True)
rel = float(np.max(np.abs(a[f] - b[f]) / np.maximum(np.abs(a[f]), 1e-300))) if f.any() else 0.0
print('A vs $v logliks: bitwise' if same else f'A vs $v: differ, max rel {rel:.3e}')
"; done
rm -f "$OUT"/*.npy
exit $rc
