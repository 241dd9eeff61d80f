#!/bin/bash
# TVλ GPU pass: the TVλ / edge / states GPU tests, then config-3 benches (certified, FP64) and
# optionally the selective-certification probe.  Each GPU step has its own time limit; the chain
# stops at the first failure.   usage: bash tools/archive/r3_tvl.sh <tag> [probe]
set -eo pipefail
export TMPDIR=/tmp
TAG=${1:-tvl}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
rc=0; timeout -k 10 300 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_edge.py tests/test_gpu_states.py -m gpu -v -s --timeout 120 --timeout-method thread > "$OUT/pytest_tvl.log" 2>&1 || rc=$?
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" "$OUT/pytest_tvl.log" | head -30 || true; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stop"; exit 1; fi
tail -2 "$OUT/pytest_tvl.log"
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
python -c "import json; d=json.load(open('$OUT/bench_c3.json')); print('c3 cert', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline'].get('parity'))"
timeout -k 10 200 python -u bench.py --config 3 --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/bench_c3_fp64.json" 2> "$OUT/bench_c3_fp64.err"
python -c "import json; d=json.load(open('$OUT/bench_c3_fp64.json')); print('c3 fp64', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
if [ "${2:-}" = "probe" ]; then
  timeout -k 10 300 python -u tools/tvl_detect_probe.py "$OUT/probe.npz"
fi
if [ -f tools/libyfm_old.so ] && [ "${3:-}" = "old" ]; then
  YFM_LIB=tools/libyfm_old.so timeout -k 10 200 python -u -m pytest tests/test_gpu_tvl.py -m gpu -v --timeout 120 --timeout-method thread -k "1024" > "$OUT/pytest_old.log" 2>&1 || true
  grep -E "certified 1024|fp64 1024|passed|failed" "$OUT/pytest_old.log" || true
  YFM_LIB=tools/libyfm_old.so timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/bench_c3_old.json" 2> "$OUT/bench_c3_old.err"
  python -c "import json; d=json.load(open('$OUT/bench_c3_old.json')); print('c3 cert OLD', d['value'], d['roofline']['kernel_ms'])"
fi
