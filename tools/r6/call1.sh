#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c1
mkdir -p $O
timeout -k 10 120 ./tools/empty_launch_probe > $O/empty_launch.txt 2>&1 || exit 1
cat $O/empty_launch.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_deferred.py -x -q --timeout 120 --timeout-method thread > $O/pytest_deferred.log 2>&1 || { tail -20 $O/pytest_deferred.log; exit 1; }
tail -2 $O/pytest_deferred.log
bash tools/r6/abn.sh $O/ab20 3 "olddd nodd" --config 2 --steps 20 --warmup 5 || exit 1
bash tools/r6/abn.sh $O/ab200 2 "olddd nodd" --config 2 --steps 200 --warmup 20 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-host-rate --steps 50 > $O/kt_bench.json 2> $O/kt.err || exit 1
cat $O/kt/*/run_kernel_stats.csv 2>/dev/null | head -5 || find $O/kt -name "*stats*"
