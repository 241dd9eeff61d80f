#!/bin/bash
# Round 5: the steady-state gates after the mean-path gain cap (yfm_fixedz.hpp contraction_bound), plus the
# config-2 driver command and configs 4/5 (the cap must not cost the benchmark class its frozen waves).
set -u
O=gpurun_out/r5/${1:-steady}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py -m gpu -v -rA --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/pytest_steady.log 2>&1
rc=$?
tail -3 $O/pytest_steady.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 4
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-rate > $O/bench_c2.json 2> $O/bench_c2.err || exit 5
timeout -k 10 300 python bench.py --config 4 --steps 30 --warmup 5 --no-cpu-baseline --no-host-rate > $O/bench_c4.json 2> $O/bench_c4.err || exit 6
echo "done rc_pytest=$rc"
