#!/bin/bash
# FP64 TVλ at L ≥ 16: the propagation's products split over the quads of a row (in-tree) vs the previous kernel
# (prevfp): TVλ GPU tests, then FP64 B = 1 and B = 1,024 (L = 64), logliks compared bitwise
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c32
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_edge.py tests/test_gpu_predict.py tests/test_gpu_states.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc = 0 ] || exit 1
bash tools/r6/abn.sh $O/b1 3 "prevfp" --config 3 --batch 1 --precision fp64 --steps 30 --warmup 3 || exit 1
bash tools/r6/abn.sh $O/b1024 2 "prevfp" --config 3 --batch 1024 --precision fp64 --steps 30 --warmup 3 || exit 1
