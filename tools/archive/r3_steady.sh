#!/bin/bash
# Frozen-covariance steady state of the DNS kernel: its tests, then config 2 / 4 benches with it on and off.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-steady}
mkdir -p "$OUT"
rc=0; timeout -k 10 400 python -u -m pytest tests/test_gpu_steady.py tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_estimate.py -m gpu -v -s --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || rc=$?
grep -E "^FAILED|passed|failed|steady vs full" "$OUT/pytest.log" | tail -15 || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stop"; exit 1; fi
for S in 1 0 1; do
  YFM_DNS_STEADY=$S timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-rate > "$OUT/c2_s$S.json" 2> "$OUT/c2_s$S.err"
  python -c "import json; d=json.load(open('$OUT/c2_s$S.json')); print('c2 steady=$S', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
for S in 1 0; do
  YFM_DNS_STEADY=$S timeout -k 10 200 python -u bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/c4_s$S.json" 2> "$OUT/c4_s$S.err"
  python -c "import json; d=json.load(open('$OUT/c4_s$S.json')); print('c4 steady=$S', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_cmd.json" 2> "$OUT/driver_cmd.err"
python -c "import json; d=json.load(open('$OUT/driver_cmd.json')); print('driver cmd', d['value'], d['ms_per_step'])"
