#!/bin/bash
# DNS z̃ scratch in the planar layout (no LDS bank conflicts) vs the committed build: config 2 alternated,
# bitwise comparison of the logliks, LDS counters of both, the DNS steady/parity tests on the new one.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab7}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
NEW=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
for v in base new; do
  lib=variants/libyfm_base.so; [ $v = new ] && lib=$NEW
  YFM_LIB=$lib timeout -k 10 200 python -u tools/bitwise_dump.py "$OUT/ll_$v.npz" > "$OUT/dump_$v.log" 2>&1; ok
done
python -c "
import numpy as np
a=np.load('$OUT/ll_base.npz'); b=np.load('$OUT/ll_new.npz')
for k in a.files: print(k, 'bitwise equal' if np.array_equal(a[k], b[k], equal_nan=True) else 'DIFFERENT')
"
for rep in 1 2 3; do
  for v in base new; do
    lib=variants/libyfm_base.so; [ $v = new ] && lib=$NEW
    YFM_LIB=$lib timeout -k 10 200 python -u bench.py --config 2 --no-cpu-baseline --no-host-rate \
      > "$OUT/c2_${v}_$rep.json" 2> "$OUT/c2_${v}_$rep.err"; ok
    python -c "import json; d=json.load(open('$OUT/c2_${v}_$rep.json')); print('c2 $v rep $rep', d['value'], d['roofline']['kernel_ms'])"
  done
done
for v in base new; do
  lib=variants/libyfm_base.so; [ $v = new ] && lib=$NEW
  YFM_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$OUT/pmc_$v" -o p --output-format csv -- python3 bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate \
    > "$OUT/pmc_$v.log" 2>&1; ok
  python tools/pmc_summary.py "$OUT"/pmc_$v/*counter_collection.csv > "$OUT/pmc_$v.txt" 2>&1; ok
  grep -E "fixedz_loglik|LDS|WAIT" "$OUT/pmc_$v.txt" | cut -c1-240 | head -20
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_streams.py -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; exit $rc
