#!/bin/bash
# Build a timing-probe variant of libyfm_hip.so (never the product library) into scratch/probe<N>/:
#   YFM_TVL_PROBE=1  the TVλ kernels' 4×4 capacitance update replaced by a data-dependent no-op
#   YFM_TVL_PROBE=2  the FP64 TVλ kernel counts, in the throw flag, the filters whose capacitance LU ever exchanges rows
# usage: bash tools/archive/build_probe.sh 1   → then YFM_LIB=scratch/probe1/libyfm_hip.so python bench.py ...
set -eo pipefail
N=${1:-1}
OUT=scratch/probe$N
mkdir -p $OUT
for s in yieldfactormodels.jl_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -DYFM_TVL_PROBE=$N -c $s -o $OUT/$(basename $s .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUT/*.o -o $OUT/libyfm_hip.so
echo "built $OUT/libyfm_hip.so"
