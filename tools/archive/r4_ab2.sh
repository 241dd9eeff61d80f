#!/bin/bash
# Same-box A/B: config 2 with the round-3 library (variants/libyfm_r3.so) and the in-tree one (PIPE on /
# off); config 3 certified + FP64 with variants/libyfm_base.so (before the loop prefetch) and the
# in-tree one; then the whole -m gpu suite on the in-tree library.  Stops at a fault.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab2}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
NEW=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
b() {  # tag lib env... -- bench args
  local tag=$1 lib=$2; shift 2
  env YFM_LIB=$lib "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err"
}
for rep in 1 2; do
  YFM_LIB=variants/libyfm_r3.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-rate > "$OUT/c2_r3_$rep.json" 2> "$OUT/c2_r3_$rep.err"; ok
  YFM_LIB=$NEW timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-rate > "$OUT/c2_new_$rep.json" 2> "$OUT/c2_new_$rep.err"; ok
  YFM_DNS_PIPE=0 YFM_LIB=$NEW timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-rate > "$OUT/c2_newnopipe_$rep.json" 2> "$OUT/c2_newnopipe_$rep.err"; ok
  for v in r3 new newnopipe; do
    python -c "import json; d=json.load(open('$OUT/c2_${v}_$rep.json')); print('c2 $v rep $rep', d['value'], d['roofline']['kernel_ms'], (d.get('steady_state') or {}).get('frac_of_filter_steps'))"
  done
done
for rep in 1 2; do
  for v in base new; do
    lib=variants/libyfm_base.so; [ $v = new ] && lib=$NEW
    for prec in certified fp64; do
      YFM_LIB=$lib timeout -k 10 200 python -u bench.py --config 3 --steps 30 --warmup 5 --precision $prec \
        --no-cpu-baseline --no-host-rate > "$OUT/c3_${prec}_${v}_$rep.json" 2> "$OUT/c3_${prec}_${v}_$rep.err"; ok
      python -c "import json; d=json.load(open('$OUT/c3_${prec}_${v}_$rep.json')); print('c3 $v $prec rep $rep', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
    done
  done
done
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread --maxfail=20 \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -30
tail -2 "$OUT/pytest_gpu.log"
exit $rc
