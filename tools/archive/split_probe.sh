#!/bin/bash
# Split-kernel probe: role layouts and PMC passes (VALU busy / waits / LDS).
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-split_probe}
mkdir -p "$OUT"
for il in 0 1; do
  YFM_SPLIT_INTERLEAVE=$il timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-host-rate > "$OUT/c2_il$il.json" 2> "$OUT/c2_il$il.err"
  python -c "import json; d=json.load(open('$OUT/c2_il$il.json')); print('il=$il', d['value'], d['roofline']['kernel_ms'])"
done
YFM_DNS_SPLIT=0 timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-host-rate > "$OUT/c2_perlane.json" 2> /dev/null
python -c "import json; d=json.load(open('$OUT/c2_perlane.json')); print('perlane', d['value'], d['roofline']['kernel_ms'])"
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_WAVES SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $pass -d "$OUT/pmc_$n" -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > "$OUT/pmc_$n.log" 2>&1
  YFM_DNS_SPLIT=0 timeout -s KILL 90 rocprofv3 --pmc $pass -d "$OUT/pmcpl_$n" -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > "$OUT/pmcpl_$n.log" 2>&1
done
python tools/pmc_summary.py --kernel split_kernel "$OUT"/pmc_*/*counter_collection.csv > "$OUT/pmc_split.json" || true
python tools/pmc_summary.py --kernel fixedz_loglik "$OUT"/pmcpl_*/*counter_collection.csv > "$OUT/pmc_perlane.json" || true
cat "$OUT/pmc_split.json" "$OUT/pmc_perlane.json"
