#!/bin/bash
# Round-5 DNS setup/store changes, config 2 (and config 4): in-tree (A: σ-permuted rows + early chunk loads)
# against each one turned off (B), then the DNS parity/steady tests on the in-tree library.
set -u
O=gpurun_out/r5/sigma; mkdir -p $O
for v in r4base nosigma noearly; do
  bash tools/ab_run.sh $v $O/ab_$v --config 2 --steps 200 --warmup 20 > $O/ab_$v.txt 2>&1 || exit 1
done
bash tools/ab_run.sh r4base $O/ab_r4base_c4 --config 4 --steps 20 --warmup 3 > $O/ab_r4base_c4.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_edge.py tests/test_gpu_states.py tests/test_gpu_workloads.py > $O/pytest.log 2>&1
