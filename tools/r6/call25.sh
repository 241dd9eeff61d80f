#!/bin/bash
# the table-driven dd_exp (in-tree) vs the Taylor-and-squarings one (prev): certified tests, config 3, B = 1, the TVλ
# re-estimation
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/${C25:-c25}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_edge.py tests/test_gpu_deferred.py tests/test_gpu_predict.py tests/test_gpu_estimate.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc = 0 ] || exit 1
bash tools/r6/abn.sh $O/c3_cert 2 "prev" --config 3 --steps 10 --warmup 2 || exit 1
bash tools/r6/abn.sh $O/b1_cert 2 "prev" --config 3 --batch 1 --steps 20 --warmup 3 || exit 1
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so
for v in A prev; do
  if [ $v = A ]; then cp $O/.libA.so $LIB; else cp tools/variants/prev.so $LIB; fi
  timeout -k 10 300 python -u tools/bench_estimate.py --model tvl --no-cpu --no-cpu-opt > $O/est_tvl_$v.json 2> $O/est_tvl_$v.err || { cp $O/.libA.so $LIB; tail $O/est_tvl_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/est_tvl_$v.json')); print('est tvl $v', d['gpu_seconds_all_windows'], d['gpu_objective_evals'], d['ll_median'])"
done
cp $O/.libA.so $LIB; rm -f $O/.libA.so
