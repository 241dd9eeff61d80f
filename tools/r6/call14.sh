#!/bin/bash
# FP64 TVλ: the LDS prefetch of the one-jump loop (in-tree) vs without it (nopf) vs the committed kernel (tvlhead)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c14
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_edge.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc = 0 ] || exit 1
bash tools/r6/abn.sh $O/b1_fp64 2 "nopf tvlhead" --config 3 --batch 1 --precision fp64 --steps 40 --warmup 5 || exit 1
bash tools/r6/abn.sh $O/c3_fp64 2 "nopf tvlhead" --config 3 --precision fp64 --steps 20 --warmup 3 || exit 1
bash tools/r6/abn.sh $O/b1024_fp64 1 "nopf tvlhead" --config 3 --batch 1024 --precision fp64 --steps 40 --warmup 5 || exit 1
