#!/bin/bash
# Targeted GPU pass: selected -m gpu tests, then one default bench line (with the CPU baseline).
# usage: bash tools/archive/r3_quick.sh <tag> "<pytest -k expr>" [bench args...]
set -eo pipefail
export TMPDIR=/tmp
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread --maxfail=30 -k "$K" > "$OUT/pytest_gpu.log" 2>&1 || echo "pytest failed"
grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -40
if [ "$#" -gt 0 ] || [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
  python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['outputs'], json.dumps(d.get('cpu_baseline') or {})[:1500])"
fi
