#!/bin/bash
# A/B of the in-tree library (A) against tools/variants/<tag>.so (B), alternated on one box.
# usage: bash tools/ab_run.sh <tag> <out-dir> <bench args...>   (e.g. --config 3 --steps 20 --warmup 3)
# Each bench runs under its own time limit; the in-tree library is restored at the end.
set -u
TAG=$1; OUT=$2; shift 2
mkdir -p "$OUT"
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp "$LIB" "$OUT/.libA.so"
rc=0
for rep in 1 2; do
  for v in A B; do
    if [ $v = B ]; then cp "tools/variants/$TAG.so" "$LIB"; else cp "$OUT/.libA.so" "$LIB"; fi
    YFM_BENCH_DUMP="$OUT/$v$rep.npy" timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-host-rate > "$OUT/$v$rep.json" 2> "$OUT/$v$rep.err" || { rc=$?; break 2; }
    python -c "import json; d=json.load(open('$OUT/$v$rep.json')); print('$v$rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
cp "$OUT/.libA.so" "$LIB"
rm -f "$OUT/.libA.so"
# the logliks of A and B (same workload, same seed): bitwise, or the largest relative difference
[ $rc = 0 ] && python -c "
import numpy as np
a, b = np.load('$OUT/A1.npy'), np.load('$OUT/B1.npy')
f = np.isfinite(a) & np.isfinite(b)
same = np.array_equal(a, b, equal_nan=True)
rel = float(np.max(np.abs(a[f] - b[f]) / np.maximum(np.abs(a[f]), 1e-300))) if f.any() else 0.0
print('A vs B logliks: bitwise' if same else f'A vs B logliks: differ, max rel {rel:.3e}, finite A/B {np.isfinite(a).sum()}/{np.isfinite(b).sum()}')
"
rm -f "$OUT"/*.npy
exit $rc
