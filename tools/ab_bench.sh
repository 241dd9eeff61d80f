mkdir -p gpurun_out/ab
for lib in new old; do
  if [ $lib = old ]; then export YFM_LIB=$PWD/yieldfactormodels.jl_amd/yfm_amd/libyfm_hip_old.so; else unset YFM_LIB; fi
  for c in 2 5; do
    timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/${lib}_c$c.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab/${lib}_c$c.json').read().splitlines()[-1]);print('$lib c$c', d['value'], d['roofline']['kernel_ms'])"
  done
done
