#!/bin/bash
# The driver's bench command on the final build (twice), then the config-2 PMC passes.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-drv}
mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_cmd_$i.json" 2> "$OUT/driver_cmd_$i.err"
  python -c "import json; d=json.load(open('$OUT/driver_cmd_$i.json')); print('driver cmd', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
EVALS=65536 STEPS=599 bash tools/pmc_config.sh 2 "$OUT/pmc_c2"
