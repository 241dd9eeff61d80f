#!/bin/bash
# TVλ A/B on one box: config 3 certified and FP64 with variants/libyfm_base.so (before) and the in-tree
# library (after), alternated, then the TVλ GPU tests on the in-tree library.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4tvl}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
NEW=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
for rep in 1 2; do
  for v in base new; do
    lib=variants/libyfm_base.so; [ $v = new ] && lib=$NEW
    for prec in certified fp64; do
      YFM_LIB=$lib timeout -k 10 200 python -u bench.py --config 3 --steps 30 --warmup 5 --precision $prec \
        --no-cpu-baseline --no-host-rate > "$OUT/c3_${prec}_${v}_$rep.json" 2> "$OUT/c3_${prec}_${v}_$rep.err"; ok
      python -c "import json; d=json.load(open('$OUT/c3_${prec}_${v}_$rep.json')); print('$v $prec rep $rep', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('parity', {}))" | cut -c1-400
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_tvl.py -v -s --timeout 300 --timeout-method thread > "$OUT/pytest_tvl.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest_tvl.log" | tail -30
exit $rc
