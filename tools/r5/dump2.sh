#!/bin/bash
set -u
O=gpurun_out/r5/dump2
mkdir -p $O
timeout -k 10 200 python tools/r5/dump_case2.py --find > $O/find.log 2>&1 || exit 1
B=$(python -c "import ast;l=open('$O/find.log').read().split('worst ')[1];print(ast.literal_eval(l.strip())[0][0])")
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so
for v in dumpA dumpB; do
  cp tools/variants/$v.so $LIB
  timeout -k 10 200 python tools/r5/dump_case2.py --dump $B > $O/$v.log 2>&1 || { cp $O/.libA.so $LIB; exit 2; }
done
cp $O/.libA.so $LIB; rm -f $O/.libA.so
echo ok $B
