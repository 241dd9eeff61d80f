#!/bin/bash
# Round-5 GNS5: A fragments pinned in AGPRs for the 4×4×4 MFMAs (in-tree, A) vs not (B), config 5, bitwise
# compare; then the GNS5 tests.
set -u
O=gpurun_out/r5/gns_agpr; mkdir -p $O
bash tools/ab_run.sh nognsagpr $O/ab_nognsagpr --config 5 --steps 10 --warmup 3 > $O/ab_nognsagpr.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_workloads.py tests/test_gpu_states.py tests/test_gpu_deferred.py tests/test_gpu_split_form.py > $O/pytest.log 2>&1
