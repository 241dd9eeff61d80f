# Estimator timing under env variants (via gpurun): bash tools/est_ab.sh
mkdir -p gpurun_out/est
run() { tag=$1; shift
  env YFM_EST_STATS=1 "$@" timeout -k 10 120 python -u tools/bench_estimate.py --no-cpu > gpurun_out/est/$tag.json 2> gpurun_out/est/$tag.err || exit 1
  echo "$tag: $(grep -o '"gpu_seconds_all_windows": [0-9.]*' gpurun_out/est/$tag.json) $(grep 'rounds' gpurun_out/est/$tag.err | tail -1)"
}
run zc_g2 YFM_EST_GROUPS=2 YFM_EST_ZEROCOPY=1
run zc_g1 YFM_EST_GROUPS=1 YFM_EST_ZEROCOPY=1
run dma_g1 YFM_EST_GROUPS=1 YFM_EST_ZEROCOPY=0
run dma_g2 YFM_EST_GROUPS=2 YFM_EST_ZEROCOPY=0
run zc_g2b YFM_EST_GROUPS=2 YFM_EST_ZEROCOPY=1
