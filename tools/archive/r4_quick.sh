#!/bin/bash
# Targeted GPU pass: selected -m gpu tests (pytest -k), then one bench line.
# Stops at a fault / abort / timeout (exit status other than 0 or 1 from pytest); plain test failures
# (status 1) still run the bench.
# usage: bash tools/archive/r4_quick.sh <tag> "<pytest -k expr>" [bench args...]     (NOBENCH=1: skip the bench)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread --maxfail=30 -k "$K" \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -60
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "bench exit $rc"; tail -20 "$OUT/bench.err"; exit $rc; fi
  python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['outputs'], json.dumps(d.get('steady_state') or {})[:600], json.dumps(d.get('cpu_baseline') or {})[:800])"
fi
