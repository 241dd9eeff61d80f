#!/bin/bash
# a randomised (SEEDS cases, default 1,000) parity sweep on the final round-6 build (tests/test_gpu_random.py with YFM_RANDOM_SEEDS)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c26
mkdir -p $O
rm -f $O/sweep.jsonl
YFM_RANDOM_SEEDS=${SEEDS:-1000} YFM_SWEEP_REPORT=$O/sweep.jsonl timeout -k 10 1080 python -u -m pytest tests/test_gpu_random.py -k test_random_cases_vs_c_oracle -v --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
python - <<PY
import json
rows = [json.loads(l) for l in open("$O/sweep.jsonl")]
print("cases", len(rows), "finite candidates", sum(r["n"] for r in rows), "strict failures", sum(len(r["strict_fail"]) for r in rows),
      "within only by term scale", sum(len(r["within_only_by_term_scale"]) for r in rows))
PY
exit $rc
