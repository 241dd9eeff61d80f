#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/r6/tests.sh t1 || exit 1
bash tools/r6/abn.sh gpurun_out/r6/ab_pf 2 "pf" --config 3 --steps 10 --warmup 2 || exit 1
O=gpurun_out/r6/emu
mkdir -p $O
for c in 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --emulate-world 8 --steps 20 --warmup 3 > $O/c${c}_w8.json 2> $O/c${c}_w8.err || exit 1
  python -c "import json; d=json.load(open('$O/c${c}_w8.json')); print($c, d['predicted_efficiency'], d['max_rank_kernel_ms'], d['world1']['kernel_ms_mean'], d['rank_imbalance'])"
done
