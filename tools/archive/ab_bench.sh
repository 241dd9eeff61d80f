# A/B of the in-tree library against yfm_amd/libyfm_hip_old.so on the given configs.
# usage (via gpurun): bash tools/archive/ab_bench.sh "2 5" [steps]
mkdir -p gpurun_out/ab
CONFIGS=${1:-"2 5"}
STEPS=${2:-100}
for lib in new old new; do
  if [ $lib = old ]; then export YFM_LIB=$PWD/yieldfactormodels.jl_amd/yfm_amd/libyfm_hip_old.so; else unset YFM_LIB; fi
  for c in $CONFIGS; do
    timeout -k 10 200 python -u bench.py --config $c --steps $STEPS --warmup 10 --no-cpu-baseline > gpurun_out/ab/${lib}_c$c.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab/${lib}_c$c.json').read().splitlines()[-1]);print('$lib c$c', d['value'], d['roofline']['kernel_ms'])"
  done
done
