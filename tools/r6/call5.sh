#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c5
mkdir -p $O
timeout -k 10 120 ./tools/fp64_dep_probe > $O/fp64_dep_probe.txt 2>&1 || exit 1
cat $O/fp64_dep_probe.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_estimate.py -x -v -s --timeout 200 --timeout-method thread > $O/pytest_tvl.log 2>&1; rc=$?
grep -E "power mode|passed|failed|FAILED|Error" $O/pytest_tvl.log | tail -12
[ $rc = 0 ] || exit 1
YFM_EST_STATS=1 timeout -k 10 300 python -u tools/bench_estimate.py --model tvl --no-cpu --no-cpu-opt > $O/est_tvl.json 2> $O/est_tvl.err || { tail $O/est_tvl.err; exit 1; }
python -c "import json; d=json.load(open('$O/est_tvl.json')); print('tvl est', d['gpu_seconds_all_windows'], d['gpu_objective_evals'])"
tail -3 $O/est_tvl.err
bash tools/r6/abn.sh $O/ab_c3 1 "" --config 3 --steps 10 --warmup 2 || exit 1
