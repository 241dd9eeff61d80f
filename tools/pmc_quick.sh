set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
timeout -k 10 200 python -u bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pmc2/c2.json
python -c "import json;d=json.loads(open('gpurun_out/pmc2/c2.json').read().splitlines()[-1]);print('c2', d['value'], d['roofline']['kernel_ms'])"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d gpurun_out/pmc2/p -o p --output-format csv -- python3 bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc2/p.log 2>&1
python tools/pmc_summary.py gpurun_out/pmc2/p/*counter_collection.csv
