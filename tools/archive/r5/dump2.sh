#!/bin/bash
set -u
O=gpurun_out/r5/dump2
mkdir -p $O
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so
cp tools/variants/dumpA.so $LIB
timeout -k 10 200 python tools/r5/dump_case2.py --find > $O/find.log 2>&1 || { cp $O/.libA.so $LIB; exit 1; }
B=$(python -c "import ast;l=open('$O/find.log').read().split('worst ')[1];print(ast.literal_eval(l.strip().splitlines()[0])[0][0])")
for v in dumpA dumpB; do
  cp tools/variants/$v.so $LIB
  timeout -k 10 200 python tools/r5/dump_case2.py --dump $B > $O/$v.log 2>&1 || { cp $O/.libA.so $LIB; exit 2; }
done
cp $O/.libA.so $LIB; rm -f $O/.libA.so
timeout -k 10 600 python tools/c4_parity_scan.py > $O/c4_scan.json 2> $O/c4_scan.err || exit 3
echo ok $B
