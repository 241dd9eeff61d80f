#!/bin/bash
# Config-2 kernel time and instruction counts, round-3 library vs the in-tree one: rocprofv3 kernel stats
# (50 timed steps) and one PMC pass of VALU / LDS counters each.  Every step under its own hard limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4prof1}
mkdir -p "$OUT"
NEW=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
for v in r3 new; do
  lib=variants/libyfm_r3.so; [ $v = new ] && lib=$NEW
  export YFM_LIB=$lib
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kt_$v" -o kt --output-format csv -- \
    python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host-rate > "$OUT/kt_$v.json" 2> "$OUT/kt_$v.err" || exit $?
  f=$(find "$OUT/kt_$v" -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "fixedz|Name" "$f" | cut -d, -f1-8
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU \
    -d "$OUT/pmc_$v" -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > "$OUT/pmc_$v.log" 2>&1 || exit $?
  f=$(find "$OUT/pmc_$v" -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'EOF'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    k = r.get("Kernel_Name", "")
    if "fixedz_loglik" not in k: continue
    agg[r["Counter_Name"]][r.get("Dispatch_Id", "")] += float(r["Counter_Value"])
for c, d in sorted(agg.items()):
    vals = list(d.values()); print(f"  {c:26s} per dispatch {sum(vals)/len(vals):.4e} ({len(vals)} dispatches)")
EOF
done
