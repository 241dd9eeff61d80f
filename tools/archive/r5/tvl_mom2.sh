#!/bin/bash
set -u
O=gpurun_out/r5/${1:-tvl_mom2}
mkdir -p $O
bash tools/r5/dump.sh || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_states.py tests/test_gpu_edge.py tests/test_gpu_random.py \
  tests/test_gpu_predict.py tests/test_gpu_estimate.py -m gpu -v -rA --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_tvl.log 2>&1
rc=$?
tail -3 $O/pytest_tvl.log
[ $rc -le 1 ] || exit $rc
bash tools/ab_run.sh tvl_basis $O/ab_c3 --config 3 --steps 20 --warmup 3 --settle-seconds 0.3 || exit 8
echo "done rc_pytest=$rc"
