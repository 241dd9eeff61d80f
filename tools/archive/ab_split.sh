#!/bin/bash
# A/B of the DNS kernels: the two-wave split (default) vs one filter per lane (YFM_DNS_SPLIT=0):
# bitwise test, then config-2 / config-4 benches of both, then a rocprofv3 kernel-stats pass.
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab_split}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -v --timeout 200 --timeout-method thread > "$OUT/pytest_split.log" 2>&1 || { echo "split test failed"; grep -E "^E |FAILED" "$OUT/pytest_split.log" | head -20; }
tail -2 "$OUT/pytest_split.log"
for mode in 0 1; do
  YFM_DNS_SPLIT=$mode timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-rate > "$OUT/c2_split$mode.json" 2> "$OUT/c2_split$mode.err"
  python -c "import json; d=json.load(open('$OUT/c2_split$mode.json')); print('c2 split=$mode', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  YFM_DNS_SPLIT=$mode timeout -k 10 200 python -u bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/c4_split$mode.json" 2> "$OUT/c4_split$mode.err"
  python -c "import json; d=json.load(open('$OUT/c4_split$mode.json')); print('c4 split=$mode', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-rate > "$OUT/traced.json" 2> "$OUT/prof.err"
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
head -5 "$OUT/kernel_stats.csv" | cut -c1-200
