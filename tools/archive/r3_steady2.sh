#!/bin/bash
# Full GPU suite, config-2/4 benches (steady state on; the bench reports the full-recursion rate beside
# it), the driver's own command, and PMC passes of the config-2 kernel.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-steady}
mkdir -p "$OUT"
rc=0; timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
grep -E "^FAILED|passed|failed|steady vs full" "$OUT/pytest_gpu.log" | tail -15 || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stop"; exit 1; fi
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
python -c "import json; d=json.load(open('$OUT/bench_c2.json')); r=d['roofline']; s=d['steady_state']; print('c2', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], 'steady frac', s['frac_of_filter_steps'], 'full', s['full_recursion_evals_per_s'], s['full_recursion_kernel_ms'], s['vs_full_recursion_max_rel'], d['cpu_baseline']['parity'])"
timeout -k 10 300 python -u bench.py --config 4 --steps 30 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
python -c "import json; d=json.load(open('$OUT/bench_c4.json')); r=d['roofline']; s=d['steady_state']; print('c4', d['value'], r['kernel_ms'], r['frac'], s['frac_of_filter_steps'], s['full_recursion_kernel_ms'], s['vs_full_recursion_max_rel'])"
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_cmd.json" 2> "$OUT/driver_cmd.err"
python -c "import json; d=json.load(open('$OUT/driver_cmd.json')); print('driver cmd', d['value'], d['ms_per_step'])"
EVALS=65536 STEPS=599 bash tools/pmc_config.sh 2 "$OUT/pmc_c2"
