#!/bin/bash
# bench.py with sampled per-launch events (every 8th): config 2 default and the driver's command, rocprofv3
# kernel statistics of the same command, the multi-rank bench tests.
set -u
export TMPDIR=/tmp
O=gpurun_out/r5/ev2; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-rate > $O/kt_c2.json 2> $O/kt_c2.err || exit 1
find $O/kt_c2 -name "*kernel_trace.csv" -delete
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_multirank.py > $O/pytest_multirank.log 2>&1
