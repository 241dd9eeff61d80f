#!/bin/bash
# Round-5 σ-permuted MFMA rows (16-byte z̃ stores) — in-tree (A) vs YFM_DNS_SIGMA=0 (B) and vs σ + look-ahead,
# config 2; then the DNS parity/steady tests on the in-tree library.
set -u
O=gpurun_out/r5/sigma; mkdir -p $O
bash tools/ab_run.sh nosigma $O/ab_nosigma --config 2 --steps 200 --warmup 20 > $O/ab_nosigma.txt 2>&1 || exit 1
bash tools/ab_run.sh la $O/ab_la --config 2 --steps 200 --warmup 20 > $O/ab_la.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_steady_sweep.py tests/test_gpu_steady.py tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_edge.py tests/test_gpu_states.py > $O/pytest.log 2>&1
