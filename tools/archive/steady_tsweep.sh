#!/bin/bash
# Config-2 kernel time against the panel length T (B = 65,536): the slope is the per-step cost of the
# steady block, the intercept the setup + the first (full-recursion) blocks.
set -eo pipefail
OUT=gpurun_out/${1:-tsweep}
mkdir -p "$OUT"
for T in 34 66 130 258 600; do
  for s in 1 0; do
    YFM_DNS_STEADY=$s timeout -k 10 200 python -u bench.py --T $T --steps 100 --warmup 10 --no-cpu-baseline --no-host-rate > "$OUT/T${T}_s$s.json" 2> "$OUT/T${T}_s$s.err"
    python -c "import json; d=json.load(open('$OUT/T${T}_s$s.json')); print('T $T steady $s', d['roofline']['kernel_ms'])"
  done
done
