#!/bin/bash
# Round-5 DNS: A fragments read by the MFMAs straight from AGPRs (in-tree, A) against the copies (noagpr),
# against the mid-block switch off (nomid) and against the round-4 kernel (r4base), config 2 (+4), bitwise
# compare; the MFMA-block micro probe; the phase probe; the DNS tests.
set -u
O=gpurun_out/r5/agpr; mkdir -p $O
timeout -k 10 60 ./tools/mfma_block_probe > $O/mfma_block_probe.txt 2>&1 || exit 1
for v in noagpr nomid r4base; do
  bash tools/ab_run.sh $v $O/ab_$v --config 2 --steps 200 --warmup 20 > $O/ab_$v.txt 2>&1 || exit 1
done
bash tools/ab_run.sh r4base $O/ab_r4base_c4 --config 4 --steps 20 --warmup 3 > $O/ab_r4base_c4.txt 2>&1 || exit 1
YFM_LIB=tools/variants/ph.so timeout -k 10 200 python -u tools/phase_run.py > $O/phase_ph.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_edge.py tests/test_gpu_states.py tests/test_gpu_workloads.py > $O/pytest.log 2>&1
