#!/bin/bash
# Round 5: certified TVλ in the moment basis — the TVλ parity tests, then A/B against the loading basis.
set -u
O=gpurun_out/r5/tvl_mom
mkdir -p $O
bash tools/r5/steady.sh steady2 || exit $?
timeout -k 10 240 python tools/dbg_c4_steady.py > gpurun_out/r5/steady2/dbg_c4.log 2>&1 || exit 7
timeout -k 10 600 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_states.py tests/test_gpu_edge.py tests/test_gpu_random.py \
  tests/test_gpu_predict.py -m gpu -v -rA --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_tvl.log 2>&1
rc=$?
tail -3 $O/pytest_tvl.log
[ $rc -le 1 ] || exit $rc
bash tools/ab_run.sh tvl_basis $O/ab_c3 --config 3 --steps 20 --warmup 3 --settle-seconds 0.3 || exit 8
echo "done rc_pytest=$rc"
