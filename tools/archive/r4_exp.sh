#!/bin/bash
# Same-box timing A/B of config 2 over variant libraries (tools/archive/exp_variant.sh), alternated twice.
#   bash tools/archive/r4_exp.sh <tag> <lib-name> [<lib-name> ...]     (lib-name: a variants/libyfm_<name>.so, or "new")
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for v in "$@"; do
    lib=variants/libyfm_$v.so; [ "$v" = new ] && lib=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
    [ "$v" = newnopipe ] && lib=yieldfactormodels.jl_amd/yfm_amd/libyfm_hip.so
    pipe=1; [ "$v" = newnopipe ] && pipe=0
    YFM_DNS_PIPE=$pipe YFM_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-rate ${BENCH_ARGS} \
      > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || { echo "bench $v failed"; tail -5 "$OUT/${v}_$rep.err"; exit 3; }
    python -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); print('$v rep $rep', d['value'], d['roofline']['kernel_ms'], d['ms_per_step'], (d.get('steady_state') or {}).get('frac_of_filter_steps'))"
  done
done
