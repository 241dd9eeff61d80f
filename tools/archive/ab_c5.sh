#!/bin/bash
# GNS5 (config 5) timing over several library builds + the GNS5 GPU tests on the first:
# bash tools/archive/ab_c5.sh <tag> <lib.so>...
set -eo pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp "$LIB" "$OUT/.libA.so"
cp "$1" "$LIB"
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || echo "pytest failed"
tail -2 "$OUT/pytest.log"
for l in "$@"; do
  n=$(basename "$l" .so)
  cp "$l" "$LIB"
  timeout -k 10 200 python -u bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/c5_$n.json" 2> "$OUT/c5_$n.err"
  python -c "import json; d=json.load(open('$OUT/c5_$n.json')); print('c5 $n', d['value'], d['roofline']['kernel_ms'])"
done
cp "$OUT/.libA.so" "$LIB"
rm -f "$OUT/.libA.so"
