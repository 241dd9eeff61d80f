#!/bin/bash
# Round-5 DNS: the first row-tile group's z̃ stores interleaved with the second group's MFMAs (in-tree, A) vs back
# to back (noil), configs 2 and 4, bitwise compare; then the DNS tests.
set -u
O=gpurun_out/r5/il; mkdir -p $O
bash tools/ab_run.sh noil $O/ab_noil --config 2 --steps 200 --warmup 20 > $O/ab_noil.txt 2>&1 || exit 1
bash tools/ab_run.sh noil $O/ab_noil_c4 --config 4 --steps 20 --warmup 3 > $O/ab_noil_c4.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_edge.py tests/test_gpu_states.py tests/test_gpu_workloads.py > $O/pytest.log 2>&1
