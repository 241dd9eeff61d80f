#!/bin/bash
# PMC passes of the config-3 kernels (certified and FP64) + an FP64 group-width probe.
set -eo pipefail
export TMPDIR=/tmp
EVALS=16384 STEPS=599 bash tools/pmc_config.sh 3 gpurun_out/pmc_r3/c3_certified
EVALS=16384 STEPS=599 bash tools/pmc_config.sh 3 gpurun_out/pmc_r3/c3_fp64 --precision fp64
for L in 4 8 16; do
  YFM_TVL_LANES=$L timeout -k 10 200 python -u bench.py --config 3 --precision fp64 --steps 30 --warmup 5 --no-cpu-baseline --no-host-rate > gpurun_out/pmc_r3/c3_fp64_L$L.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/pmc_r3/c3_fp64_L$L.json')); print('fp64 L=$L', d['roofline']['kernel_ms'])"
done
