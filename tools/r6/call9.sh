#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c9
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_multirank.py -x -v -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|passed|failed|predicted" $O/pytest.log | tail -30
[ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_estimate.py --model tvl --precision fp64 --no-cpu --no-cpu-opt > $O/est_tvl_fp64.json 2> $O/est_tvl_fp64.err || { tail $O/est_tvl_fp64.err; exit 1; }
python -c "import json; d=json.load(open('$O/est_tvl_fp64.json')); print('tvl fp64 est', d['gpu_seconds_all_windows'], d['gpu_objective_evals'], d['ll_median'])"
