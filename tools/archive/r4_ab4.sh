#!/bin/bash
# The dd init fused into the dd loglik kernel: configs 2 and 5 with variants/libyfm_base.so vs the in-tree
# library, alternated; then the deferral / random-sweep / edge tests on the in-tree library.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ab4}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
NEW=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
for rep in 1 2; do
  for v in base new; do
    lib=variants/libyfm_base.so; [ $v = new ] && lib=$NEW
    for c in 2 5; do
      steps=200; [ $c = 5 ] && steps=20
      YFM_LIB=$lib timeout -k 10 200 python -u bench.py --config $c --steps $steps --warmup 5 --no-cpu-baseline --no-host-rate \
        > "$OUT/c${c}_${v}_$rep.json" 2> "$OUT/c${c}_${v}_$rep.err"; ok
      python -c "import json; d=json.load(open('$OUT/c${c}_${v}_$rep.json')); print('c$c $v rep $rep', d['value'], d['roofline']['kernel_ms'])"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_random.py tests/test_gpu_edge.py tests/test_gpu_large_n.py \
  -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "FAILED|ERROR" "$OUT/pytest.log" | head; tail -1 "$OUT/pytest.log"
exit $rc
