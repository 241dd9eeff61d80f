#!/bin/bash
# Round-5 DNS: the (4, 2, 2) tile grouping is the default — the DNS/GNS5 GPU tests on it and a bench line.
set -u
O=gpurun_out/r5/il2t; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_edge.py tests/test_gpu_states.py tests/test_gpu_workloads.py tests/test_gpu_deferred.py tests/test_gpu_split.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
