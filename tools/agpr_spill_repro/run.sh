#!/bin/bash
# Run the reproducer on a GPU box (build it first on the CPU: python tools/agpr_spill_repro/build.py).
# Both libraries are built from commit 13e51a6's sources (the last build without the fence) with the same
# flags except `-mllvm -amdgpu-spill-vgpr-to-agpr=0`.  Expected with ROCm 7.2: the fenced build gives 0
# differing candidates between the two update forms, the unfenced one O(1)-wrong two-function logliks
# (DESIGN.md §5).  Also runs the shipped library (HEAD).  Exit 0 iff the fenced builds agree.
set -u
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
CASE="$HERE/case2431.bin"
timeout -k 10 60 "$HERE/repro" "$HERE/build/libyfm_13e51a6_fenced.so" "$CASE" || exit 1
timeout -k 10 60 "$HERE/repro" "$HERE/build/libyfm_13e51a6_unfenced.so" "$CASE"
unfenced=$?
[ "$unfenced" -le 1 ] || exit 1
timeout -k 10 60 "$HERE/repro" "$ROOT/yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so" "$CASE" || exit 1
echo "13e51a6 unfenced: exit $unfenced (1 = the miscompile reproduced: the forms differ; 0 = this ROCm agrees)"
