#!/bin/bash
# DNS MFMA-phase experiments vs the committed build (variants/libyfm_<v>.so): row tiles per accumulator group
# (rg4, rg2), the block's NaN flags read before the MFMAs (enan); bitwise checks, config 2 alternated, and the
# phase-timing probes (phase: committed layout; phrg4: with 4 row tiles per group).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab9}
VARS=${VARS:-"base rg4 rg2 enan"}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
for v in $VARS; do
  YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u tools/bitwise_dump.py "$OUT/ll_$v.npz" > "$OUT/dump_$v.log" 2>&1; ok
done
python -c "
import numpy as np
a=np.load('$OUT/ll_base.npz')
for v in '$VARS'.split()[1:]:
    b=np.load('$OUT/ll_%s.npz' % v)
    print(v, [(k, 'bitwise equal' if np.array_equal(a[k], b[k], equal_nan=True) else 'DIFFERENT') for k in a.files])
"
for rep in 1 2 3; do
  for v in $VARS; do
    YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u bench.py --config 2 --no-cpu-baseline --no-host-rate \
      > "$OUT/c2_${v}_$rep.json" 2> "$OUT/c2_${v}_$rep.err"; ok
    python -c "import json; d=json.load(open('$OUT/c2_${v}_$rep.json')); print('c2 $v rep $rep', d['value'], d['roofline']['kernel_ms'])"
  done
done
for v in ${PROBES:-phase phrg4}; do
  YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u tools/phase_run.py > "$OUT/$v.log" 2>&1; ok
  echo "== $v"; sed -n '/timed launch/,$p' "$OUT/$v.log" | head -6
done
