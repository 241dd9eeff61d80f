#!/bin/bash
# Round-6 evidence pass on the committed build (one GPU call): the whole -m gpu suite, smoke, and per config 2-5
# the PMC passes (one counter group per run, each under a hard limit) with their per-kernel summary, the
# rocprofv3 kernel statistics and the bench line (which reads the PMC summary for roofline.traffic); config 3 at
# B = 1 and 1,024 with their own PMC passes; the emulated 8-GPU shards of configs 4 and 5; the rolling
# re-estimation benchmarks; the driver's own bench command.
#   bash tools/r6/final.sh <outdir under gpurun_out/>   (SKIP_TESTS=1: no pytest/smoke; CONFIGS="2 3": those
#   configurations only; SKIP_EXTRA=1: no small-B / emulation / estimator / driver-command steps)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6final}
mkdir -p "$OUT"
timeout -k 5 60 rocm-smi --showclocks --showpower --showtemp > "$OUT/smi_before.txt" 2>&1 || true
ok() { local rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread --maxfail=20 \
    > "$OUT/pytest_gpu.log" 2>&1; ok
  grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -20; tail -1 "$OUT/pytest_gpu.log"
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; ok
  tail -1 "$OUT/smoke.log"
fi
pmc() {  # pmc <dir> <evals> <bench args...>: the four counter passes of one launch size, then their summary
  local P=$1 ev=$2; shift 2
  mkdir -p "$P"
  pass() { name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$P/$name" -o $name --output-format csv -- \
      python3 bench.py "${ARGS[@]}" --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > "$P/$name.log" 2>&1
  }
  ARGS=("$@")
  pass fetch FETCH_SIZE || return $?
  pass write WRITE_SIZE || return $?
  pass valu SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES || return $?
  pass stall SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || return $?
  python3 tools/pmc_summary.py --evals $ev --steps 599 $(find "$P" -name "*counter_collection.csv") > "$P/pmc_summary.json" || return 3
  find "$P" -name "*counter_collection.csv" -size +2M -delete
}
declare -A EV=([2]=65536 [3]=16384 [4]=983040 [5]=1048576)
for c in ${CONFIGS:-2 3 4 5}; do
  pmc "$OUT/pmc_c$c" ${EV[$c]} --config $c || { echo "pmc c$c failed"; exit 4; }
  # the summary where bench.py looks for it (profiles/), so this call's bench lines carry roofline.traffic
  mkdir -p profiles/r6/final/pmc_c$c && cp "$OUT/pmc_c$c/pmc_summary.json" profiles/r6/final/pmc_c$c/
  echo "pmc c$c ok"
  steps=30; [ $c = 2 ] && steps=200
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_c$c" -o kt --output-format csv -- \
    python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate > "$OUT/kt_c$c.json" 2> "$OUT/kt_c$c.err"; ok
  find "$OUT/kt_c$c" -name "*kernel_trace.csv" -delete
  timeout -k 10 300 python -u bench.py --config $c --steps $steps --warmup 5 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"; ok
  python3 -c "import json; d=json.load(open('$OUT/bench_c$c.json')); r=d['roofline']; print('c$c', d['value'], r['kernel_ms'], r['frac'], r['traffic'])"
done
[ -n "$SKIP_EXTRA" ] && exit 0
# config 3 at the estimator's batch sizes (B ∈ {1, 1,024, 16,384}): counters, kernel statistics, bench line
for B in 1 1024; do
  pmc "$OUT/pmc_c3_B$B" $B --config 3 --batch $B || { echo "pmc c3 B$B failed"; exit 4; }
  mkdir -p profiles/r6/final/pmc_c3_B$B && cp "$OUT/pmc_c3_B$B/pmc_summary.json" profiles/r6/final/pmc_c3_B$B/
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_c3_B$B" -o kt --output-format csv -- \
    python3 bench.py --config 3 --batch $B --steps 20 --warmup 3 --no-cpu-baseline --no-host-rate > "$OUT/kt_c3_B$B.json" 2> "$OUT/kt_c3_B$B.err"; ok
  find "$OUT/kt_c3_B$B" -name "*kernel_trace.csv" -delete
  timeout -k 10 300 python -u bench.py --config 3 --batch $B --steps 30 --warmup 5 > "$OUT/bench_c3_B$B.json" 2> "$OUT/bench_c3_B$B.err"; ok
  python3 -c "import json; d=json.load(open('$OUT/bench_c3_B$B.json')); print('c3 B=$B', d['value'], d['roofline']['kernel_ms'])"
done
for c in 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --emulate-world 8 --steps 20 --warmup 3 > "$OUT/emulate_c${c}_w8.json" 2> "$OUT/emulate_c${c}_w8.err"; ok
  python3 -c "import json; d=json.load(open('$OUT/emulate_c${c}_w8.json')); print('c$c w8', d['predicted_efficiency'])"
done
timeout -k 10 400 python -u tools/bench_estimate.py > "$OUT/bench_estimate.json" 2> "$OUT/bench_estimate.err"; ok
timeout -k 10 500 python -u tools/bench_estimate.py --model tvl --windows 240 > "$OUT/bench_estimate_tvl.json" 2> "$OUT/bench_estimate_tvl.err"; ok
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_cmd.json" 2> "$OUT/driver_cmd.err"; ok
timeout -k 5 60 rocm-smi --showclocks --showpower --showtemp > "$OUT/smi_after.txt" 2>&1 || true
