# Estimator timing under env variants (via gpurun): bash tools/archive/est_ab.sh tag "ENV=.. ENV=.." ...
TAG=${1:-est}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in "$@"; do
  tag=$(echo "$v" | tr -c 'A-Za-z0-9=\n' '_' | sed 's/YFM_//g')
  env YFM_EST_STATS=1 $v timeout -k 10 120 python -u tools/bench_estimate.py --no-cpu > $OUT/$tag.json 2> $OUT/$tag.err || exit 1
  echo "$v: $(grep -o '"gpu_seconds_all_windows": [0-9.]*' $OUT/$tag.json) $(grep 'rounds' $OUT/$tag.err | tail -1)"
done
