#!/bin/bash
# A/B of two library builds: A = yfm_amd/libyfm_hip.so (in tree), B = tools/libyfm_hip_B.so.
# usage: bash tools/archive/ab_lib.sh <tag> [pytest -k expr]
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab_lib}
mkdir -p "$OUT"
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp "$LIB" "$OUT/.libA.so"
if [ -n "$2" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "$2" > "$OUT/pytest_A.log" 2>&1 || echo "pytest A failed"
  tail -2 "$OUT/pytest_A.log"
fi
for rep in 1 2; do
  for v in A B; do
    if [ $v = B ]; then cp tools/libyfm_hip_B.so "$LIB"; else cp "$OUT/.libA.so" "$LIB"; fi
    timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-rate > "$OUT/c2_$v$rep.json" 2> "$OUT/c2_$v$rep.err"
    python -c "import json; d=json.load(open('$OUT/c2_$v$rep.json')); print('c2 $v$rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
for v in A B; do
  if [ $v = B ]; then cp tools/libyfm_hip_B.so "$LIB"; else cp "$OUT/.libA.so" "$LIB"; fi
  timeout -k 10 200 python -u bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/c4_$v.json" 2> "$OUT/c4_$v.err"
  python -c "import json; d=json.load(open('$OUT/c4_$v.json')); print('c4 $v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
cp "$OUT/.libA.so" "$LIB"
rm -f "$OUT/.libA.so"
