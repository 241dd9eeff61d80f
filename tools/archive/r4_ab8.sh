#!/bin/bash
# DNS z̃ scratch swizzled (XOR + pair swap, conflict-free b64 stores and b128 reads) vs the committed build:
# bitwise check, config 2 alternated, LDS counters; a phase-timing probe; steady/parity/stream tests on swz.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab8}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
for v in base swz; do
  YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u tools/bitwise_dump.py "$OUT/ll_$v.npz" > "$OUT/dump_$v.log" 2>&1; ok
done
python -c "
import numpy as np
a=np.load('$OUT/ll_base.npz'); b=np.load('$OUT/ll_swz.npz')
for k in a.files: print(k, 'bitwise equal' if np.array_equal(a[k], b[k], equal_nan=True) else 'DIFFERENT')
"
for rep in 1 2 3; do
  for v in base swz; do
    YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u bench.py --config 2 --no-cpu-baseline --no-host-rate \
      > "$OUT/c2_${v}_$rep.json" 2> "$OUT/c2_${v}_$rep.err"; ok
    python -c "import json; d=json.load(open('$OUT/c2_${v}_$rep.json')); print('c2 $v rep $rep', d['value'], d['roofline']['kernel_ms'])"
  done
done
YFM_LIB=variants/libyfm_swz.so timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d "$OUT/pmc_swz" -o p --output-format csv -- python3 bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate \
  > "$OUT/pmc_swz.log" 2>&1; ok
python tools/pmc_summary.py "$OUT"/pmc_swz/*counter_collection.csv > "$OUT/pmc_swz.txt" 2>&1; ok
grep -E "fixedz_loglik|LDS" "$OUT/pmc_swz.txt" | head -8
YFM_LIB=variants/libyfm_phase.so timeout -k 10 200 python -u tools/phase_run.py > "$OUT/phase.log" 2>&1; ok
sed -n '/timed launch/,$p' "$OUT/phase.log" | head -20
YFM_LIB=variants/libyfm_swz.so timeout -k 10 600 python -u -m pytest tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_streams.py -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; exit $rc
