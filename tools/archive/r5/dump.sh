#!/bin/bash
set -u
O=gpurun_out/r5/dump
mkdir -p $O
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so
for v in dumpA dumpB; do
  cp tools/variants/$v.so $LIB
  timeout -k 10 120 python tools/r5/dump_case.py > $O/$v.log 2>&1 || { cp $O/.libA.so $LIB; exit 1; }
done
cp $O/.libA.so $LIB; rm -f $O/.libA.so
echo ok
