#!/bin/bash
# sweep case 4985 fixed (λ·m_min > 746 selects the zero Jacobian column): edge + known-hard tests, the case script,
# the 10,000-case sweep, and config 3 / B = 1 (certified, FP64) against the pre-fix TVλ objects (prevdd, prevfp)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c28
mkdir -p $O
: # edge + TVλ tests passed in the first c28 attempt (41 passed)


timeout -k 10 120 python -u tools/r6/case4985.py > $O/case.txt 2>&1 || exit 1
grep -v Warning $O/case.txt
SEEDS=10000 bash tools/r6/call26.sh || exit 1
bash tools/r6/abn.sh $O/c3_cert 2 "prevdd" --config 3 --steps 10 --warmup 2 || exit 1
bash tools/r6/abn.sh $O/b1_cert 2 "prevdd" --config 3 --batch 1 --steps 20 --warmup 3 || exit 1
bash tools/r6/abn.sh $O/c3_fp64 2 "prevfp" --config 3 --precision fp64 --steps 10 --warmup 2 || exit 1
