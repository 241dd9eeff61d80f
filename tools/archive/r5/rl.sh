#!/bin/bash
# Round-5 DNS: a whole steady block's chunk rotation deferred to the next block's start (rl) vs after its steps
# (in-tree); configs 2 and 4 with a bitwise compare, then the DNS tests on the rl library.
set -u
O=gpurun_out/r5/rl; mkdir -p $O
bash tools/ab_run.sh rl $O/ab_rl --config 2 --steps 200 --warmup 20 > $O/ab_rl.txt 2>&1 || exit 1
bash tools/ab_run.sh rl $O/ab_rl_c4 --config 4 --steps 20 --warmup 3 > $O/ab_rl_c4.txt 2>&1 || exit 1
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so && cp tools/variants/rl.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_edge.py tests/test_gpu_workloads.py tests/test_gpu_deferred.py > $O/pytest_rl.log 2>&1; rc=$?
cp $O/.libA.so $LIB; rm -f $O/.libA.so
exit $rc
