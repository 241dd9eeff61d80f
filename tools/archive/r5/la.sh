#!/bin/bash
# Round-5 look-ahead MFMA A/B (DNS config 2) + the nowrite store-tail bound, then the steady/parity tests on the
# look-ahead library.
set -u
O=gpurun_out/r5/la; mkdir -p $O
bash tools/ab_run.sh nowrite $O/ab_nowrite --config 2 --steps 200 --warmup 20 > $O/ab_nowrite.txt 2>&1 || exit 1
bash tools/ab_run.sh la $O/ab_la --config 2 --steps 200 --warmup 20 > $O/ab_la.txt 2>&1 || exit 1
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so && cp tools/variants/la.so $LIB
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_random.py > $O/pytest_la.log 2>&1; rc=$?
cp $O/.libA.so $LIB; rm -f $O/.libA.so
exit $rc
