#!/bin/bash
# sweep case 4985 (TVλ, N = 12, T = 3): the current library and the session-start TVλ objects (start.so)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c27
mkdir -p $O
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so
timeout -k 10 120 python -u tools/r6/case4985.py > $O/current.txt 2>&1; rc=$?
cat $O/current.txt | grep -v Warning
cp tools/variants/start.so $LIB
timeout -k 10 120 python -u tools/r6/case4985.py > $O/start.txt 2>&1; rc2=$?
cp $O/.libA.so $LIB; rm -f $O/.libA.so
echo "--- start.so"; cat $O/start.txt | grep -v Warning
[ $rc = 0 ] && [ $rc2 = 0 ]
