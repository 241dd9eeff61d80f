#!/bin/bash
# a wider randomised trajectory sweep (predict + get_loss_array vs the oracle / binary128 truth) on the final build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c34
mkdir -p $O
YFM_TRAJ_SEEDS=${SEEDS:-600} timeout -k 10 900 python -u -m pytest tests/test_gpu_random.py -k test_random_trajectories_vs_oracle -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
exit $rc
