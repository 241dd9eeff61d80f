#!/bin/bash
set -u
O=gpurun_out/r5/micro
mkdir -p $O
timeout -k 10 120 ./tools/fp64_waves > $O/fp64_waves.txt 2>&1 || exit 1
cat $O/fp64_waves.txt
YFM_GNS5_STEADY=1 timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate > $O/c5_steady.json 2> $O/c5_steady.err || exit 2
python -c "import json; d=json.load(open('$O/c5_steady.json')); print('c5 steady', d['value'], d['roofline']['kernel_ms'], d['steady_state']['frac_of_filter_steps'], d['steady_state']['full_recursion_kernel_ms'])"
