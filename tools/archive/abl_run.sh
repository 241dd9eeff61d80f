#!/bin/bash
# Ablation timing of the DNS steady kernel (probe build tools/libyfm_abl.so; YFM_ABL bits: 2 = no MFMA
# block in steady blocks, 4 = no steady math, 8 = no NaN scan).  Results are timing-only.
set -eo pipefail
OUT=gpurun_out/${1:-abl}
mkdir -p "$OUT"
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp tools/libyfm_hip_B.so "$LIB"
for a in 0 2 4 6 8 14; do
  YFM_ABL=$a timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-rate > "$OUT/c2_$a.json" 2> "$OUT/c2_$a.err" || true
  if [ $a = 0 ]; then cp tools/libyfm_abl.so "$LIB"; YFM_ABL=0 timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-rate > "$OUT/c2_abl0.json" 2> "$OUT/c2_abl0.err"; fi
done
for f in "$OUT"/c2_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['roofline']['kernel_ms'], d.get('steady_state',{}).get('share'))" || true; done
cp tools/libyfm_hip_B.so "$LIB"
