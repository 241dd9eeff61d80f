#!/bin/bash
# FP64 TVλ (config 3) timing over several library builds: bash tools/archive/ab_tvl_fp64.sh <tag> <lib.so>...
set -eo pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp "$LIB" "$OUT/.libA.so"
for rep in 1 2; do
  for l in "$@"; do
    n=$(basename "$l" .so)
    cp "$l" "$LIB"
    timeout -k 10 200 python -u bench.py --config 3 --precision fp64 --steps 30 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/c3f_${n}_$rep.json" 2> "$OUT/c3f_${n}_$rep.err"
    python -c "import json; d=json.load(open('$OUT/c3f_${n}_$rep.json')); print('c3 fp64 $n $rep', d['value'], d['roofline']['kernel_ms'])"
  done
done
cp "$OUT/.libA.so" "$LIB"
rm -f "$OUT/.libA.so"
