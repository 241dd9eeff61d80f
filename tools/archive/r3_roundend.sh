#!/bin/bash
# Round-end rehearsal on the committed build: the -m gpu suite, smoke(), the driver's default bench.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-roundend}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
python -c "import json; d=json.load(open('$OUT/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
python -c "import json; d=json.load(open('$OUT/bench_c5.json')); s=d.get('steady_state') or {}; print('c5', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], s.get('frac_of_filter_steps'), s.get('full_recursion_kernel_ms'), s.get('vs_full_recursion_max_rel'))"
