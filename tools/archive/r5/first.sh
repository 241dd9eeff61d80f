#!/bin/bash
# Round 5, first GPU pass: the GPU suite (new: de-aliased steady sweep + DNS NaN thaw cases, two-rank driver),
# the AGPR-spill reproducer, the driver's bench command, config 3 at B = 1 / 1,024 with a lane-width sweep,
# and the TVλ rolling re-estimation.  Output: gpurun_out/r5/first/.
set -u
O=gpurun_out/r5/first
mkdir -p $O
rocm-smi --showclocks --showpower > $O/smi_start.txt 2>&1 || true
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
timeout -k 10 180 bash tools/agpr_spill_repro/run.sh > $O/agpr_repro.log 2>&1; rr=$?
tail -2 $O/agpr_repro.log
[ $rr -le 1 ] || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 4
for B in 1 1024; do
  for L in 4 8 16 32 64; do
    YFM_TVL_LANES=$L timeout -k 10 300 python bench.py --config 3 --batch $B --steps 20 --warmup 3 --no-cpu-baseline \
      --no-host-rate --settle-seconds 0.2 > $O/c3_B${B}_L${L}.json 2> $O/c3_B${B}_L${L}.err || exit 5
  done
done
echo "c3 sweep done"
timeout -k 10 400 python tools/bench_estimate.py --model tvl --windows 240 > $O/est_tvl.json 2> $O/est_tvl.err || exit 6
echo "all done rc_pytest=$rc"
