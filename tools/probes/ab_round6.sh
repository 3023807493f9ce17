# Round 6's last A/B runs (tools/ab.sh): 6 waves per SIMD for small trees (-DSRT_GW_SMALL=6 build)
cd /root/repo
export STEPS=5 REPEAT=2
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_gw6_knot bash tools/ab.sh "base|" "gw6|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_gw6.so" && \
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_gw6_air bash tools/ab.sh "base|" "gw6|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_gw6.so" && \
SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_gw6.so timeout -k 10 120 python tools/probes/gw5_block.py
