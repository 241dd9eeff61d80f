#!/bin/bash
# power mode with the squarings shared per step (in-tree) vs dd_powi per power (prevdd): TVλ
# re-estimation (240 windows, N = 30), estimator GPU tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c33
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_estimate.py tests/test_gpu_tvl.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc = 0 ] || exit 1
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so
for v in A prevdd A prevdd; do
  if [ $v = A ]; then cp $O/.libA.so $LIB; else cp tools/variants/$v.so $LIB; fi
  timeout -k 10 300 python -u tools/bench_estimate.py --model tvl --no-cpu --no-cpu-opt > $O/est_tvl_$v.json 2> $O/est_tvl_$v.err || { cp $O/.libA.so $LIB; tail $O/est_tvl_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/est_tvl_$v.json')); print('est tvl $v', d['gpu_seconds_all_windows'], d['gpu_objective_evals'], d['ll_median'])"
done
cp $O/.libA.so $LIB; rm -f $O/.libA.so
