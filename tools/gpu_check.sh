#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats.  Each GPU step
# has its own time limit and the chain stops at the first failure.
# usage (from the repo root, via gpurun): bash tools/gpu_check.sh [tag]
set -eo pipefail
export TMPDIR=/tmp
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
echo "pytest ok"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "smoke ok"
timeout -k 10 200 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > "$OUT/bench_traced.json" 2> "$OUT/prof.err"
echo "rocprof ok"
