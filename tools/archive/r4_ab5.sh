#!/bin/bash
# Certified TVλ: variants/libyfm_base.so vs the in-tree library (z2-sums accumulated as u = (1 − z)/m),
# alternated; then the TVλ GPU tests (1,024-candidate truth sample, states, windows) on the in-tree one.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab5}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
NEW=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
for rep in 1 2; do
  for v in base new; do
    lib=variants/libyfm_base.so; [ $v = new ] && lib=$NEW
    YFM_LIB=$lib timeout -k 10 200 python -u bench.py --config 3 --steps 30 --warmup 5 --no-cpu-baseline --no-host-rate \
      > "$OUT/c3_${v}_$rep.json" 2> "$OUT/c3_${v}_$rep.err"; ok
    python -c "import json; d=json.load(open('$OUT/c3_${v}_$rep.json')); print('c3 $v rep $rep', d['value'], d['roofline']['kernel_ms'])"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_states.py -v -s --timeout 300 --timeout-method thread \
  > "$OUT/pytest_tvl.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|certified 1024" "$OUT/pytest_tvl.log" | cut -c1-300 | head; tail -1 "$OUT/pytest_tvl.log"
exit $rc
