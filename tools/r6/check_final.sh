#!/bin/bash
# the round-end driver's steps on the committed build: pytest -m gpu, smoke, bench.py defaults
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6/check_final
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['metric'], d['value'], d['ms_per_step'], d['roofline']['frac'])"
