#!/bin/bash
# certified TVλ latency mode: the 1/λ factoring at L = 64 (in-tree) vs prev, repeated
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c23
mkdir -p $O
bash tools/r6/abn.sh $O/b1_cert 3 "prev" --config 3 --batch 1 --steps 20 --warmup 3 || exit 1
bash tools/r6/abn.sh $O/b1024_cert 2 "prev" --config 3 --batch 1024 --steps 20 --warmup 3 || exit 1
