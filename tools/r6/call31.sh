#!/bin/bash
# certified TVλ at L ≥ 16: u split over the quads (in-tree) vs the previous kernel (prevdd); TVλ GPU tests, then
# B = 1 and B = 1,024 (L = 64) and a forced L = 16 config-3 run, logliks
# compared bitwise
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/${C31:-c31}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_edge.py tests/test_gpu_predict.py tests/test_gpu_states.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc = 0 ] || exit 1
bash tools/r6/abn.sh $O/b1 3 "prevdd" --config 3 --batch 1 --steps 20 --warmup 3 || exit 1
bash tools/r6/abn.sh $O/b1024 2 "prevdd" --config 3 --batch 1024 --steps 20 --warmup 3 || exit 1
YFM_TVL_LANES=16 bash tools/r6/abn.sh $O/c3_l16 1 "prevdd" --config 3 --batch 4096 --steps 5 --warmup 1 || exit 1
