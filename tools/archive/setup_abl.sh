#!/bin/bash
# Setup-cost ablation of the DNS loglik kernel (probe build tools/libyfm_sabl.so, timing only; YFM_ABL
# bits: 16 = no Lyapunov start, 32 = no fragment staging, 64 = no loading exps), full recursion, T = 34.
set -eo pipefail
OUT=gpurun_out/${1:-sabl}
mkdir -p "$OUT"
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp "$LIB" "$OUT/.libA.so"
cp tools/libyfm_sabl.so "$LIB"
for a in 0 16 32 64 112; do
  for T in 2 34; do
    YFM_DNS_STEADY=0 YFM_ABL=$a timeout -k 10 200 python -u bench.py --T $T --steps 100 --warmup 10 --no-cpu-baseline --no-host-rate > "$OUT/a${a}_T$T.json" 2> "$OUT/a${a}_T$T.err" || true
    python -c "import json; d=json.load(open('$OUT/a${a}_T$T.json')); print('abl $a T $T', d['roofline']['kernel_ms'])" || true
  done
done
cp "$OUT/.libA.so" "$LIB"
rm -f "$OUT/.libA.so"
