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
    timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-host-rate > "$OUT/$v$rep.json" 2> "$OUT/$v$rep.err" || { rc=$?; break 2; }
    python -c "import json; d=json.load(open('$OUT/$v$rep.json')); print('$v$rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
cp "$OUT/.libA.so" "$LIB"
rm -f "$OUT/.libA.so"
exit $rc
