#!/bin/bash
# Round-5 evidence pass on the committed build (one GPU call): the whole -m gpu suite, smoke, and per
# config 2-5 the PMC passes (one counter group per run, each under a hard limit) with their per-kernel
# summary, the rocprofv3 kernel statistics, and the bench line (which reads the PMC summary for
# roofline.traffic), then the rolling re-estimation benchmark and the driver's own bench command.
#   bash tools/r5/final.sh <outdir under gpurun_out/>      (SKIP_TESTS=1: no pytest/smoke; CONFIGS="2 3": those
#   configurations only; SKIP_EXTRA=1: no small-B / estimator / probe / driver-command steps)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5final}
mkdir -p "$OUT"
# the card's clocks, power and temperature before and after (box-to-box variation: one pass ran every config
# 12-17% slower, TVλ included, whose kernel had not changed; profiles/r4/slow_box/)
timeout -k 5 60 rocm-smi --showclocks --showpower --showtemp > "$OUT/smi_before.txt" 2>&1 || true
ok() { local rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread --maxfail=20 \
    > "$OUT/pytest_gpu.log" 2>&1; ok
  grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -20; tail -1 "$OUT/pytest_gpu.log"
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; ok
  tail -1 "$OUT/smoke.log"
fi
declare -A EV=([2]=65536 [3]=16384 [4]=983040 [5]=1048576)
for c in ${CONFIGS:-2 3 4 5}; do
  P="$OUT/pmc_c$c"
  mkdir -p "$P"
  pass() { name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$P/$name" -o $name --output-format csv -- \
      python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-host-rate > "$P/$name.log" 2>&1
  }
  pass fetch FETCH_SIZE || exit $?
  pass write WRITE_SIZE || exit $?
  pass valu SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES || exit $?
  pass stall SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
  python3 tools/pmc_summary.py --evals ${EV[$c]} --steps 599 $(find "$P" -name "*counter_collection.csv") > "$P/pmc_summary.json" || exit 3
  find "$P" -name "*counter_collection.csv" -size +2M -delete
  # the summary where bench.py looks for it (profiles/), so this call's bench lines carry roofline.traffic
  mkdir -p profiles/r5/final/pmc_c$c && cp "$P/pmc_summary.json" profiles/r5/final/pmc_c$c/
  echo "pmc c$c ok"
  steps=30; [ $c = 2 ] && steps=200
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_c$c" -o kt --output-format csv -- \
    python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-rate > "$OUT/kt_c$c.json" 2> "$OUT/kt_c$c.err"; ok
  find "$OUT/kt_c$c" -name "*kernel_trace.csv" -delete
  timeout -k 10 300 python -u bench.py --config $c --steps $steps --warmup 5 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"; ok
  python3 -c "import json; d=json.load(open('$OUT/bench_c$c.json')); r=d['roofline']; print('c$c', d['value'], r['kernel_ms'], r['frac'], r['traffic'])"
done
[ -n "$SKIP_EXTRA" ] && exit 0
# config 3 at the estimator's batch sizes (B ∈ {1, 1,024, 16,384}): kernel statistics + bench line
for B in 1 1024; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_c3_B$B" -o kt --output-format csv -- \
    python3 bench.py --config 3 --batch $B --steps 20 --warmup 3 --no-cpu-baseline --no-host-rate > "$OUT/kt_c3_B$B.json" 2> "$OUT/kt_c3_B$B.err"; ok
  find "$OUT/kt_c3_B$B" -name "*kernel_trace.csv" -delete
  timeout -k 10 300 python -u bench.py --config 3 --batch $B --steps 30 --warmup 5 > "$OUT/bench_c3_B$B.json" 2> "$OUT/bench_c3_B$B.err"; ok
  python3 -c "import json; d=json.load(open('$OUT/bench_c3_B$B.json')); print('c3 B=$B', d['value'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python -u tools/bench_estimate.py > "$OUT/bench_estimate.json" 2> "$OUT/bench_estimate.err"; ok
timeout -k 10 400 python -u tools/bench_estimate.py --model tvl --windows 240 > "$OUT/bench_estimate_tvl.json" 2> "$OUT/bench_estimate_tvl.err"; ok
timeout -k 10 60 ./tools/mfma_block_probe > "$OUT/mfma_block_probe.txt" 2>&1; ok
timeout -k 10 300 bash tools/agpr_spill_repro/run.sh > "$OUT/agpr_repro.log" 2>&1; ok
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_cmd.json" 2> "$OUT/driver_cmd.err"; ok
python3 -c "import json; d=json.load(open('$OUT/driver_cmd.json')); print('driver cmd', d['value'], d['ms_per_step'])"
timeout -k 5 60 rocm-smi --showclocks --showpower --showtemp > "$OUT/smi_after.txt" 2>&1 || true
