#!/bin/bash
# The round-4 DNS build candidate (early NaN flags, 4-tile MFMA groups, two-round wave-local fragment staging)
# vs the committed build and enrg4: bitwise check, config 2 and config 5 alternated, phase probe; the DNS/GNS5
# steady, parity, sweep and workload tests on it.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab13}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
for v in base new; do
  YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u tools/bitwise_dump.py "$OUT/ll_$v.npz" > "$OUT/dump_$v.log" 2>&1; ok
done
python -c "
import numpy as np
a=np.load('$OUT/ll_base.npz'); b=np.load('$OUT/ll_new.npz')
print('new', [(k, 'bitwise equal' if np.array_equal(a[k], b[k], equal_nan=True) else 'DIFFERENT') for k in a.files])
"
for rep in 1 2 3; do
  for v in base enrg4 new; do
    YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u bench.py --config 2 --no-cpu-baseline --no-host-rate \
      > "$OUT/c2_${v}_$rep.json" 2> "$OUT/c2_${v}_$rep.err"; ok
    python -c "import json; d=json.load(open('$OUT/c2_${v}_$rep.json')); print('c2 $v rep $rep', d['value'], d['roofline']['kernel_ms'])"
  done
done
for v in base new; do
  YFM_LIB=variants/libyfm_$v.so timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --no-host-rate \
    > "$OUT/c5_${v}.json" 2> "$OUT/c5_${v}.err"; ok
  python -c "import json; d=json.load(open('$OUT/c5_${v}.json')); print('c5 $v', d['value'], d['roofline']['kernel_ms'])"
done
YFM_LIB=variants/libyfm_phnew.so timeout -k 10 200 python -u tools/phase_run.py > "$OUT/phnew.log" 2>&1; ok
sed -n '/timed launch/,$p' "$OUT/phnew.log" | head -4
YFM_LIB=variants/libyfm_new.so timeout -k 10 900 python -u -m pytest tests/test_gpu_steady.py tests/test_gpu_steady_sweep.py \
  tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_workloads.py tests/test_gpu_deferred.py -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "FAILED|ERROR" "$OUT/pytest.log" | cut -c1-200 | head; tail -2 "$OUT/pytest.log"; exit $rc
