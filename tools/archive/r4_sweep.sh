#!/bin/bash
# The 3,000-seed randomised parity sweep (tests/test_gpu_random.py) and the stream-ordering tests on the
# current build.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4sweep}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -v --timeout 120 --timeout-method thread > "$OUT/pytest_streams.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_streams.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
YFM_RANDOM_SEEDS=3000 YFM_SWEEP_REPORT=$OUT/sweep_report.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_random.py \
  -k test_random_cases_vs_c_oracle -q --timeout 300 --timeout-method thread > "$OUT/sweep3000.log" 2>&1
rc2=$?; tail -3 "$OUT/sweep3000.log"
exit $(( rc > rc2 ? rc : rc2 ))
