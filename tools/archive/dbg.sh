#!/bin/bash
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/dbg_seed.py 292 916 2431 10 > gpurun_out/dbg.log 2>&1 || true
cat gpurun_out/dbg.log | tail -40
