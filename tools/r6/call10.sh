#!/bin/bash
# GNS5 cooperative initial-state kernel: bitwise tests, then config 5 with 1 / 2 / 4 lanes per candidate
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c10
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gns5_init.py -x -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|passed|failed|finite" $O/pytest.log | tail -12
[ $rc = 0 ] || exit 1
for r in 2 4 1 4 2; do
  YFM_GNS5_INIT_LANES=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$r -o kt --output-format csv -- \
    python3 bench.py --config 5 --no-cpu-baseline --no-host-rate --steps 10 --warmup 2 > $O/bench_$r.json 2> $O/bench_$r.err || { tail $O/bench_$r.err; exit 1; }
  python - <<PY
import csv, glob, json
f = sorted(glob.glob("$O/kt_$r/**/kt_kernel_stats.csv", recursive=True))[-1]
for row in csv.DictReader(open(f)):
    if "init" in row["Name"] or "fixedz_loglik" in row["Name"]:
        print("lanes $r", row["Name"][:48], row["Calls"], float(row["AverageNs"]) / 1e6)
d = json.loads([l for l in open("$O/bench_$r.json") if l.startswith("{")][-1])
print("lanes $r value", d["value"], "ms", d["ms_per_step"], d.get("best_candidate"))
PY
done
