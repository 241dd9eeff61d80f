#!/bin/bash
# the lane model with the L ≥ 16 costs (in-tree) vs the previous model (oldmodel: the same kernels): TVλ
# re-estimation (240 windows, N = 30), estimator GPU tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c30
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_estimate.py tests/test_gpu_tvl.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc = 0 ] || exit 1
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so
for v in A oldmodel A oldmodel; do
  if [ $v = A ]; then cp $O/.libA.so $LIB; else cp tools/variants/$v.so $LIB; fi
  timeout -k 10 300 python -u tools/bench_estimate.py --model tvl --no-cpu --no-cpu-opt > $O/est_tvl_$v.json 2> $O/est_tvl_$v.err || { cp $O/.libA.so $LIB; tail $O/est_tvl_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/est_tvl_$v.json')); print('est tvl $v', d['gpu_seconds_all_windows'], d['gpu_objective_evals'], d['ll_median'])"
done
cp $O/.libA.so $LIB; rm -f $O/.libA.so
