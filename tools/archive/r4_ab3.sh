#!/bin/bash
# Certified TVλ (config 3) with the round-3 library vs the in-tree one (dd_exp on r/2⁴), alternated; the
# whole -m gpu suite; then the default bench line.  Stops at a fault.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab3}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
NEW=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
for rep in 1 2; do
  for v in r3 new; do
    lib=variants/libyfm_r3.so; [ $v = new ] && lib=$NEW
    YFM_LIB=$lib timeout -k 10 200 python -u bench.py --config 3 --steps 30 --warmup 5 --no-cpu-baseline --no-host-rate \
      > "$OUT/c3_${v}_$rep.json" 2> "$OUT/c3_${v}_$rep.err"; ok
    python -c "import json; d=json.load(open('$OUT/c3_${v}_$rep.json')); print('c3 $v rep $rep', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread --maxfail=20 \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -30
tail -2 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 3
python -c "import json; d=json.load(open('$OUT/bench.json')); print('c2 default', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
exit $rc
