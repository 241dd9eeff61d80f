#!/bin/bash
# Generic A/B of variants/libyfm_<v>.so builds (VARS, the first is the reference): bitwise check of the DNS
# logliks against the first, config 2 alternated (REPS), config 5 once each (C5=1), phase probes (PROBES), and
# the DNS/GNS5 GPU tests on TESTLIB.
#   VARS="cur unr" PROBES="phcur phunr" TESTLIB=unr bash tools/archive/r4_ab.sh <outdir under gpurun_out/>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
REF=${VARS%% *}
for v in $VARS; do
  YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u tools/bitwise_dump.py "$OUT/ll_$v.npz" > "$OUT/dump_$v.log" 2>&1; ok
done
python -c "
import numpy as np
a=np.load('$OUT/ll_$REF.npz')
for v in '$VARS'.split()[1:]:
    b=np.load('$OUT/ll_%s.npz' % v)
    print(v, [(k, 'bitwise equal' if np.array_equal(a[k], b[k], equal_nan=True) else 'DIFFERENT') for k in a.files])
"
for rep in $(seq 1 ${REPS:-3}); do
  for v in $VARS; do
    YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u bench.py --config 2 --no-cpu-baseline --no-host-rate \
      > "$OUT/c2_${v}_$rep.json" 2> "$OUT/c2_${v}_$rep.err"; ok
    python -c "import json; d=json.load(open('$OUT/c2_${v}_$rep.json')); print('c2 $v rep $rep', d['value'], d['roofline']['kernel_ms'])"
  done
done
if [ -n "$C5" ]; then
  for v in $VARS; do
    YFM_LIB=variants/libyfm_$v.so timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --no-host-rate \
      > "$OUT/c5_${v}.json" 2> "$OUT/c5_${v}.err"; ok
    python -c "import json; d=json.load(open('$OUT/c5_${v}.json')); print('c5 $v', d['value'], d['roofline']['kernel_ms'])"
  done
fi
for v in $PROBES; do
  YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u tools/phase_run.py > "$OUT/$v.log" 2>&1; ok
  echo "== $v"; sed -n '/timed launch/,$p' "$OUT/$v.log" | grep -E "^(phase|setup)" | head -4
done
if [ -n "$TESTLIB" ]; then
  TESTS=${TESTS:-"tests/test_gpu_steady.py tests/test_gpu_steady_sweep.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_workloads.py tests/test_gpu_deferred.py"}
  YFM_LIB=variants/libyfm_$TESTLIB.so timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q --maxfail=10 \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; grep -E "FAILED|ERROR" "$OUT/pytest.log" | cut -c1-200 | head; tail -2 "$OUT/pytest.log"; exit $rc
fi
