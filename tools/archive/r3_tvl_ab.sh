#!/bin/bash
# A/B of certified-TVλ library builds: accuracy on the 1,024-candidate config-3 fixture and config-3
# throughput, per library.   usage: bash tools/archive/r3_tvl_ab.sh <tag> lib1.so lib2.so ...
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tvl_ab}
shift
mkdir -p "$OUT"
for lib in "$@"; do
  n=$(basename "$lib" .so)
  YFM_LIB=$lib timeout -k 10 120 python -u tools/tvl_ab.py "$OUT/ll_$n.npz" > "$OUT/acc_$n.json"
  cat "$OUT/acc_$n.json"
  YFM_LIB=$lib timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/bench_c3_$n.json" 2> "$OUT/bench_c3_$n.err"
  python -c "import json; d=json.load(open('$OUT/bench_c3_$n.json')); print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  YFM_LIB=$lib timeout -k 10 200 python -u bench.py --config 3 --precision fp64 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$OUT/bench_c3f_$n.json" 2> "$OUT/bench_c3f_$n.err"
  python -c "import json; d=json.load(open('$OUT/bench_c3f_$n.json')); print('$n fp64', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
