#!/bin/bash
# Full round-3 GPU pass: the -m gpu suite, then benches of configs 2-5 and the estimator, then a
# rocprofv3 kernel-trace of the config-2 and config-3 benches.  Each GPU step has its own limit; the
# chain stops at a crash/timeout (pytest assertion failures are reported and the benches still run).
# usage: bash tools/archive/r3_full.sh <tag>
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-full}
mkdir -p "$OUT"
rc=0; timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" "$OUT/pytest_gpu.log" | tail -12 || true
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stop"; exit 1; fi
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
python -c "import json; d=json.load(open('$OUT/bench_c2.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
for c in 3 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 30 --warmup 5 --cpu-seconds 5 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
  python -c "import json; d=json.load(open('$OUT/bench_c$c.json')); print('c$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
timeout -k 10 200 python -u bench.py --config 3 --precision fp64 --steps 30 --warmup 5 --no-cpu-baseline > "$OUT/bench_c3_fp64.json" 2> "$OUT/bench_c3_fp64.err"
python -c "import json; d=json.load(open('$OUT/bench_c3_fp64.json')); print('c3 fp64', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 300 python -u tools/bench_estimate.py --no-cpu > "$OUT/bench_estimate.json" 2> "$OUT/bench_estimate.err"
tail -1 "$OUT/bench_estimate.json"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_c2" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --no-cpu-baseline --no-host-rate > "$GRAFT_REPO_ROOT/$OUT/prof_c2.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_c3" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --config 3 --steps 20 --warmup 5 --no-cpu-baseline --no-host-rate > "$GRAFT_REPO_ROOT/$OUT/prof_c3.log" 2>&1
echo profiles done
