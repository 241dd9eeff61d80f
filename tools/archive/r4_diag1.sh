#!/bin/bash
# Round-4 diagnostics: split-form debug (shipped + variant libraries), steady-sweep case 9, PIPE A/B on
# config 2, the MFMA/VALU overlap microbenchmark.  Each step under its own time limit; stops at a fault.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4diag1}
mkdir -p "$OUT"
ok() { local rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step exit $rc: stopping"; exit $rc; fi; }
timeout -k 10 120 python -u tools/dbg_split.py 2431 292 > "$OUT/split_shipped.log" 2>&1; ok
for v in dbg noagpr o1; do
  YFM_LIB=variants/libyfm_$v.so timeout -k 10 120 python -u tools/dbg_split.py 2431 292 > "$OUT/split_$v.log" 2>&1; ok
done
for f in "$OUT"/split_*.log; do echo "$f: $(grep -c 'differ' "$f") differing"; done
timeout -k 10 180 python -u tools/dbg_sweep_case.py 9 > "$OUT/sweep9.log" 2>&1; ok
cat "$OUT/sweep9.log" | tail -12
for pipe in 1 0; do
  YFM_DNS_PIPE=$pipe timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-rate > "$OUT/bench_c2_pipe$pipe.json" 2> "$OUT/bench_c2_pipe$pipe.err"; ok
  python -c "import json; d=json.load(open('$OUT/bench_c2_pipe$pipe.json')); print('pipe $pipe', d['value'], d['roofline']['kernel_ms'])"
done
timeout -k 10 120 ./tools/mfma_valu_overlap > "$OUT/overlap.txt" 2>&1; ok
cat "$OUT/overlap.txt"
