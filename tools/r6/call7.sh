#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c7
mkdir -p $O
bash tools/r6/abn.sh $O/ab_c3 2 "nosel xpad" --config 3 --steps 10 --warmup 2 || exit 1
bash tools/r6/abn.sh $O/ab_c3_B1 1 "nosel xpad" --config 3 --batch 1 --steps 20 --warmup 3 || exit 1
