#!/bin/bash
# TVλ latency mode (config 3, B = 1): FP64 and certified per lane width, kernel split under rocprofv3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c12
mkdir -p $O
for prec in fp64 certified; do
  for L in 64 32 16; do
    YFM_TVL_LANES=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_${prec}_$L -o kt --output-format csv -- \
      python3 bench.py --config 3 --batch 1 --precision $prec --no-cpu-baseline --no-host-rate --steps 20 --warmup 3 > $O/b_${prec}_$L.json 2> $O/b_${prec}_$L.err || { tail $O/b_${prec}_$L.err; exit 1; }
    python - <<PY
import csv, glob, json
f = sorted(glob.glob("$O/kt_${prec}_$L/**/kt_kernel_stats.csv", recursive=True))[-1]
for row in csv.DictReader(open(f)):
    if "tvl" in row["Name"]:
        print("$prec L=$L", row["Name"][:40], row["Calls"], round(float(row["AverageNs"]) / 1e3, 1), "us")
d = json.loads([l for l in open("$O/b_${prec}_$L.json") if l.startswith("{")][-1])
print("$prec L=$L ms_per_step", d["ms_per_step"])
PY
  done
done
