#!/bin/bash
# Round-5 DNS: mid-block steady switch + σ rows + early chunks (in-tree, A) against the switch off and against
# all three off (round-4 kernel), config 2 and 4, with a bitwise loglik compare; phase probes of both; tests.
set -u
O=gpurun_out/r5/mid; mkdir -p $O
for v in nomid r4base; do
  bash tools/ab_run.sh $v $O/ab_$v --config 2 --steps 200 --warmup 20 > $O/ab_$v.txt 2>&1 || exit 1
done
bash tools/ab_run.sh r4base $O/ab_r4base_c4 --config 4 --steps 20 --warmup 3 > $O/ab_r4base_c4.txt 2>&1 || exit 1
for v in ph ph4; do
  YFM_LIB=tools/variants/$v.so timeout -k 10 200 python -u tools/phase_run.py > $O/phase_$v.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_edge.py tests/test_gpu_states.py tests/test_gpu_workloads.py > $O/pytest.log 2>&1
