#!/bin/bash
# certified TVλ at L = 64 and config 3: both changes (A), the 1/λ factoring alone (fact), the unnormalised recurrence
# alone (nnz), neither (prev)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c24
mkdir -p $O
bash tools/r6/abn.sh $O/b1_cert 2 "fact nnz prev" --config 3 --batch 1 --steps 20 --warmup 3 || exit 1
bash tools/r6/abn.sh $O/c3_cert 1 "fact nnz prev" --config 3 --steps 10 --warmup 2 || exit 1
