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
import numpy as np
rows = [json.loads(l) for l in open("$O/sweep.jsonl")]
cert = [r for r in rows if not r.get("fp64")]
f64 = [r for r in rows if r.get("fp64")]
print("cases", len(cert), "finite candidates", sum(r["n"] for r in cert), "strict failures", sum(len(r["strict_fail"]) for r in cert),
      "within only by term scale", sum(len(r["within_only_by_term_scale"]) for r in cert))
if f64:
    e = np.array([x for r in f64 for x in r["e64"]]); o = np.array([x for r in f64 for x in r["e_oracle"]])
    print("TVλ FP64 mode:", len(f64), "cases", e.size, "finite candidates; rel err vs truth median %.2e p99 %.2e max %.2e;"
          " dense FP64 oracle median %.2e p99 %.2e max %.2e" % (np.median(e), np.quantile(e, 0.99), e.max(), np.median(o), np.quantile(o, 0.99), o.max()))
    for th in (1e-12, 1e-9, 1e-6):
        print("  > %.0e: FP64 mode %d, oracle %d" % (th, int((e > th).sum()), int((o > th).sum())))
    print("  FP64 mode worse than 10x the oracle's error and > 1e-12:", int(((e > 10 * o) & (e > 1e-12)).sum()))
PY
exit $rc
