#!/bin/bash
# Round-5: every path's block-end chunk rotation deferred to the next block's start (rl2) vs only a whole steady
# block's (in-tree); configs 2, 5 (and 4) with a bitwise compare, then the DNS/GNS5 tests on rl2.
set -u
O=gpurun_out/r5/rl2; mkdir -p $O
bash tools/ab_run.sh rl2 $O/ab_c5 --config 5 --steps 10 --warmup 3 > $O/ab_c5.txt 2>&1 || exit 1
bash tools/ab_run.sh rl2 $O/ab_c2 --config 2 --steps 200 --warmup 20 > $O/ab_c2.txt 2>&1 || exit 1
bash tools/ab_run.sh rl2 $O/ab_c4 --config 4 --steps 20 --warmup 3 > $O/ab_c4.txt 2>&1 || exit 1
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so && cp tools/variants/rl2.so $LIB
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_edge.py tests/test_gpu_workloads.py tests/test_gpu_deferred.py tests/test_gpu_states.py tests/test_gpu_predict.py tests/test_gpu_split_form.py > $O/pytest_rl2.log 2>&1; rc=$?
cp $O/.libA.so $LIB; rm -f $O/.libA.so
exit $rc
