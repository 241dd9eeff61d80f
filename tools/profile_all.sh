#!/bin/bash
# One GPU-box pass over every BASELINE config: bench JSON, rocprofv3 kernel-trace stats,
# and the PMC passes (one counter group per run, each under its own hard limit) for the
# dominant kernel of configs 2, 3, 5 (skipped with NOPMC=1), then the rolling re-estimation benchmark.
# Usage (repo root, via gpurun): [NOPMC=1] bash tools/profile_all.sh [outdir]
set -eo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_all}
mkdir -p "$OUT"
for c in 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
  echo "bench c$c ok"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c$c" -o run --output-format csv -- \
    python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/traced_c$c.json" 2> "$OUT/trace_c$c.err"
  echo "trace c$c ok"
done
pass() { c=$1; name=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/pmc_c${c}_$name" -o $name --output-format csv -- \
    python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > "$OUT/pmc_c${c}_$name.log" 2>&1
  echo "pmc c$c $name ok"
}
timeout -k 10 300 python -u tools/bench_estimate.py > "$OUT/bench_estimate.json" 2> "$OUT/bench_estimate.err"
echo "bench_estimate ok"
[ -n "$NOPMC" ] && exit 0
for c in 2 3 5; do
  pass $c fetch FETCH_SIZE
  pass $c write WRITE_SIZE
  # ≤ 8 distinct SQ base counters per pass (derived counters such as SQ_INSTS_VALU_FLOPS_FP64
  # expand to several base counters: FP64 flops are computed from the valu pass instead)
  pass $c valu SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
  pass $c stall SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
done
