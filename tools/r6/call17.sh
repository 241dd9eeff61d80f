#!/bin/bash
# PMC of the FP64 TVλ kernel at B = 1 (latency mode): instructions per step, issue and wait cycles
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/c17
mkdir -p $O
pass() { name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$O/$name" -o $name --output-format csv -- \
    python3 bench.py --config 3 --batch 1 --precision fp64 --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > "$O/$name.log" 2>&1
}
pass valu SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 || exit 1
pass stall SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS || exit 1
python3 - <<PY
import csv, glob, collections
tot = collections.defaultdict(float)
for f in glob.glob("$O/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "tvl_loglik_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
# the bench ran 1 + 3 launches per pass (warmup + steps) + the fp64 side leg: report per launch via SQ_WAVES
print({k: v for k, v in sorted(tot.items())})
PY
