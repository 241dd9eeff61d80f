#!/bin/bash
# Does timing every launch with a HIP event pair cost wall time?  Config 2, alternated: events on every launch,
# every 4th, every 1000th (kernel_ms then from a sample).
set -u
O=gpurun_out/r5/events; mkdir -p $O
for rep in 1 2; do
  for e in 1 4 1000; do
    YFM_BENCH_EVENT_EVERY=$e timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host-rate > $O/e${e}_$rep.json 2> $O/e${e}_$rep.err || exit 1
    python -c "import json; d=json.load(open('$O/e${e}_$rep.json')); print('every $e', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done > $O/events.txt 2>&1
