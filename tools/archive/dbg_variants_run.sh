#!/bin/bash
# Run tools/dbg_split.py against every library in variants/ (and the shipped one); one log per library.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-variants}
mkdir -p "$OUT"
timeout -k 10 120 python -u tools/dbg_split.py > "$OUT/shipped.log" 2>&1 || exit $?
for lib in variants/libyfm_*.so; do
  n=$(basename "$lib" .so)
  YFM_LIB=$lib timeout -k 10 120 python -u tools/dbg_split.py > "$OUT/$n.log" 2>&1 || exit $?
done
for f in "$OUT"/*.log; do echo "$f: $(grep -c 'differ' "$f") differing"; done
