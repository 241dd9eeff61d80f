#!/bin/bash
# Build the host harness twice (g++ -O2, clang++ -fsanitize=memory) and run both forms of the filter on
# the 7a42719 cases (GNS5, N = 33): bitwise agreement of the two forms, and no MSan report.
set -eo pipefail
cd "$(dirname "$0")/../.."
OUT=${TMPDIR:-/tmp}/host_fixedz
mkdir -p "$OUT"
INC="-Itools/host_fixedz/stub -Iyieldfactormodels.jl_amd/csrc"
g++ -O2 -std=c++17 -ffp-contract=off $INC tools/host_fixedz/harness.cpp -o "$OUT/harness_gcc"
/opt/rocm/lib/llvm/bin/clang++ -O1 -g -std=c++17 -ffp-contract=off -fsanitize=memory -fsanitize-memory-track-origins \
  $INC tools/host_fixedz/harness.cpp -o "$OUT/harness_msan"
for seed in ${SEEDS:-292 916 2431}; do
  python tools/host_fixedz/dump_case.py "$seed" 2 "$OUT/case_$seed.bin"
  "$OUT/harness_gcc" "$OUT/case_$seed.bin" | tail -1
  "$OUT/harness_msan" "$OUT/case_$seed.bin" > "$OUT/msan_$seed.log" 2>&1 || { echo "MSan run failed:"; head -40 "$OUT/msan_$seed.log"; exit 1; }
  tail -1 "$OUT/msan_$seed.log"
done
