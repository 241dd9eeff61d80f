#!/bin/bash
# Round-5 A/B: (1) certified TVλ compiled for two waves per SIMD (≤ 256 registers: spills) at L = 8 against the
# one-wave build at L = 4 (default) and L = 8, config 3; (2) DNS first chunks issued after the θ rows (early2).
set -u
O=gpurun_out/r5/tvl2w; mkdir -p $O
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so
run() {  # tag lib lanes
  cp $2 $LIB
  YFM_TVL_LANES=$3 timeout -k 10 300 python -u bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate \
    > $O/$1.json 2> $O/$1.err || return 1
  python -c "import json; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['roofline']['kernel_ms'])"
}
for rep in 1 2; do
  run A_L4_$rep $O/.libA.so 4 || break
  run A_L8_$rep $O/.libA.so 8 || break
  run B2w_L8_$rep tools/variants/tvl2w.so 8 || break
done > $O/tvl2w.txt 2>&1
cp $O/.libA.so $LIB; rm -f $O/.libA.so
bash tools/ab_run.sh early2 $O/ab_early2 --config 2 --steps 200 --warmup 20 > $O/ab_early2.txt 2>&1
