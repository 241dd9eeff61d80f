#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
bash tools/r6/tests.sh t2 || exit 1
O=gpurun_out/r6/c4
mkdir -p $O
timeout -k 10 300 python -u bench.py --config 4 --emulate-world 8 --steps 20 --warmup 3 > $O/c4_w8.json 2> $O/c4_w8.err || exit 1
python -c "import json; d=json.load(open('$O/c4_w8.json')); print('c4 w8', d['predicted_efficiency'], d['max_rank_kernel_ms'], d['world1']['kernel_ms_mean'])"
timeout -k 10 400 python -u tools/bench_estimate.py --model tvl > $O/est_tvl.json 2> $O/est_tvl.err || { tail $O/est_tvl.err; exit 1; }
python -c "import json; d=json.load(open('$O/est_tvl.json')); print('tvl est', d['gpu_seconds_all_windows'], d['gpu_objective_evals'], d.get('cpu_optimised_seconds_all_windows'))"
timeout -k 10 400 python -u tools/bench_estimate.py > $O/est_dns.json 2> $O/est_dns.err || { tail $O/est_dns.err; exit 1; }
python -c "import json; d=json.load(open('$O/est_dns.json')); print('dns est', d['gpu_seconds_all_windows'], d['gpu_objective_evals'], d.get('cpu_optimised_seconds_all_windows'))"
