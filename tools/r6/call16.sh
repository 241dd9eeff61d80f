#!/bin/bash
# TVλ propagate from the local column with one gather (in-tree) vs the previous commit (prev)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/${C16:-c16}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_tvl.py tests/test_gpu_edge.py tests/test_gpu_predict.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc = 0 ] || exit 1
bash tools/r6/abn.sh $O/c3_cert 2 "prev" --config 3 --steps 10 --warmup 2 || exit 1
bash tools/r6/abn.sh $O/b1_cert 2 "prev" --config 3 --batch 1 --steps 20 --warmup 3 || exit 1
bash tools/r6/abn.sh $O/c3_fp64 2 "prev" --config 3 --precision fp64 --steps 20 --warmup 3 || exit 1
bash tools/r6/abn.sh $O/b1_fp64 2 "prev" --config 3 --batch 1 --precision fp64 --steps 40 --warmup 5 || exit 1
