#!/bin/bash
# DNS re-estimation: where a round's time goes (kernel durations under rocprofv3, the estimator's own host stats)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c11
mkdir -p $O
YFM_EST_STATS=1 timeout -k 10 300 python -u tools/bench_estimate.py --model dns --no-cpu --no-cpu-opt > $O/est_dns.json 2> $O/est_dns.err || { tail $O/est_dns.err; exit 1; }
tail -4 $O/est_dns.err
YFM_EST_STATS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 -u tools/bench_estimate.py --model dns --no-cpu --no-cpu-opt > $O/est_dns_kt.json 2> $O/est_dns_kt.err || { tail $O/est_dns_kt.err; exit 1; }
python - <<PY
import csv, glob, json
f = sorted(glob.glob("$O/kt/**/kt_kernel_stats.csv", recursive=True))[-1]
for row in csv.DictReader(open(f)):
    print(row["Name"][:60], row["Calls"], float(row["AverageNs"]) / 1e3, "us avg", float(row["TotalDurationNs"]) / 1e9, "s total")
for n in ("est_dns.json", "est_dns_kt.json"):
    d = json.load(open("$O/" + n))
    print(n, d["gpu_seconds_all_windows"], d["gpu_objective_evals"])
PY
