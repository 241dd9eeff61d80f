#!/bin/bash
# Round-3 GPU pass: the -m gpu suite, the 3,000-seed randomised sweep (with the |ll|-denominator
# report), then short config-2 / config-5 benches.  Each GPU step has its own time limit; the chain
# stops at the first step that fails, times out or crashes.
# usage (from the repo root, via gpurun): bash tools/archive/r3_check.sh <tag> [pytest -k expr]
set -eo pipefail
export TMPDIR=/tmp
TAG=${1:-r3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --maxfail=30 -k "$K" > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; }
else
  timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread --maxfail=30 > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; }
fi
tail -3 "$OUT/pytest_gpu.log"
rm -f "$OUT/sweep_report.jsonl"
YFM_RANDOM_SEEDS=3000 YFM_SWEEP_REPORT="$OUT/sweep_report.jsonl" timeout -k 10 300 python -u -m pytest tests/test_gpu_random.py -q --timeout 120 --timeout-method thread -k test_random_cases_vs_c_oracle > "$OUT/sweep3000.log" 2>&1 || echo "sweep failed"
tail -12 "$OUT/sweep3000.log"
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-rate > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
python -c "import json,sys; d=json.load(open('$OUT/bench_c2.json')); print('c2', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 200 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --no-host-rate > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
python -c "import json,sys; d=json.load(open('$OUT/bench_c5.json')); print('c5', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
