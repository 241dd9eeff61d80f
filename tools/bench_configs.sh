#!/bin/bash
# Every BASELINE config through bench.py on one GPU (each step under its own time limit).
set -eo pipefail
OUT=${1:-gpurun_out/configs}
mkdir -p "$OUT"
for c in 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-50} --warmup ${WARMUP:-10} > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
  cat "$OUT/bench_c$c.json"
done
