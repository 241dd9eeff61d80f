#!/bin/bash
# Round-4 GPU pass: the whole -m gpu suite, the default bench line, smoke.  Stops at a fault / abort /
# timeout (pytest exit status other than 0 or 1).
# usage: bash tools/archive/r4_full.sh <tag>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4full}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread --maxfail=20 \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -40
tail -3 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 3; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], json.dumps(d.get('steady_state') or {})[:400])"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
exit $rc
