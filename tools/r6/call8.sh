#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c8
mkdir -p $O
bash tools/r6/abn.sh $O/ab_c3 2 "w9" --config 3 --steps 10 --warmup 2 || exit 1
