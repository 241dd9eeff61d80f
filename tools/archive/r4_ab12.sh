#!/bin/bash
# Time-invariant steady mean update (YFM_DNS_TI, + early NaN flags + 4-tile MFMA groups): config 2 alternated
# with the committed build and enrg4 (early NaN + 4-tile groups only); phase probes; the DNS steady tests,
# the steady sweep and the parity tests on ti.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab12}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
for rep in 1 2 3; do
  for v in base enrg4 ti; do
    YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u bench.py --config 2 --no-cpu-baseline --no-host-rate \
      > "$OUT/c2_${v}_$rep.json" 2> "$OUT/c2_${v}_$rep.err"; ok
    python -c "import json; d=json.load(open('$OUT/c2_${v}_$rep.json')); print('c2 $v rep $rep', d['value'], d['roofline']['kernel_ms'])"
  done
done
for v in phase phti; do
  YFM_LIB=variants/libyfm_$v.so timeout -k 10 200 python -u tools/phase_run.py > "$OUT/$v.log" 2>&1; ok
  echo "== $v"; sed -n '/timed launch/,$p' "$OUT/$v.log" | grep "^phase" | head -3
done
YFM_LIB=variants/libyfm_ti.so timeout -k 10 900 python -u -m pytest tests/test_gpu_steady.py tests/test_gpu_steady_sweep.py \
  tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_random.py -x -v -s --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "max rel|steady share|FAILED|ERROR" "$OUT/pytest.log" | cut -c1-200 | head -20; tail -3 "$OUT/pytest.log"; exit $rc
