#!/bin/bash
# config 3 whole batch: the logliks of the in-tree library and of tools/variants/prev.so, saved for the truth check
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c22
mkdir -p $O
LIB=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
cp $LIB $O/.libA.so
for v in A prev; do
  if [ $v = A ]; then cp $O/.libA.so $LIB; else cp tools/variants/prev.so $LIB; fi
  YFM_BENCH_DUMP=$O/ll_$v.npy timeout -k 10 200 python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate > $O/b_$v.json 2> $O/b_$v.err || { cp $O/.libA.so $LIB; tail $O/b_$v.err; exit 1; }
done
cp $O/.libA.so $LIB; rm -f $O/.libA.so
python - <<PY
import numpy as np
a, b = np.load("$O/ll_A.npy"), np.load("$O/ll_prev.npy")
f = np.isfinite(a) & np.isfinite(b)
r = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
r[~f] = 0
idx = np.argsort(-r)[:12]
print("pattern equal", np.array_equal(np.isfinite(a), np.isfinite(b)), "n > 1e-13:", int((r > 1e-13).sum()), "n > 1e-9:", int((r > 1e-9).sum()))
for i in idx: print(i, a[i], b[i], r[i])
PY
