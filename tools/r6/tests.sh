#!/bin/bash
# GPU test suite + smoke on one box; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/${1:-tests}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc = 0 ] || { grep -n "FAILED\|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
