#!/bin/bash
# Timing A/B over several library builds: bash tools/archive/ab_multi.sh <tag> <lib.so>... (each copied in place
# of yfm_amd/libyfm_hip.so in turn; the in-tree build is restored at the end).  Optional PYTEST_K runs
# the GPU tests matching it on the first library.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp "$LIB" "$OUT/.libA.so"
if [ -n "$PYTEST_K" ]; then
  cp "$1" "$LIB"
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "$PYTEST_K" > "$OUT/pytest.log" 2>&1 || echo "pytest failed"
  tail -2 "$OUT/pytest.log"
fi
for rep in 1 2; do
  for l in "$@"; do
    n=$(basename "$l" .so)
    cp "$l" "$LIB"
    timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-rate > "$OUT/c2_${n}_$rep.json" 2> "$OUT/c2_${n}_$rep.err"
    python -c "import json; d=json.load(open('$OUT/c2_${n}_$rep.json')); print('c2 $n $rep', d['value'], d['roofline']['kernel_ms'])"
  done
done
for l in "$@"; do
  n=$(basename "$l" .so)
  cp "$l" "$LIB"
  timeout -k 10 200 python -u bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/c4_$n.json" 2> "$OUT/c4_$n.err"
  python -c "import json; d=json.load(open('$OUT/c4_$n.json')); print('c4 $n', d['value'], d['roofline']['kernel_ms'])"
done
cp "$OUT/.libA.so" "$LIB"
rm -f "$OUT/.libA.so"
