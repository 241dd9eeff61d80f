#!/bin/bash
# Certified TVλ (config 3) under LLVM's other machine schedulers, alternated with the default build; logliks
# compared bitwise.
set -u
O=gpurun_out/r5/tvl_sched; mkdir -p $O
for v in ilp memc minreg; do
  bash tools/ab_run.sh $v $O/ab_$v --config 3 --steps 10 --warmup 2 > $O/ab_$v.txt 2>&1 || exit 1
done
