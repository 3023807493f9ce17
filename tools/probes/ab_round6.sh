cd /root/repo
export STEPS=5 REPEAT=2
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_ml2_knot bash tools/ab.sh "base|" "ml2|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_ml2.so" && \
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_ml2_air bash tools/ab.sh "base|" "ml2|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_ml2.so" && \
BENCH_ARGS="--scene synthetic --synthetic-tris 1000000 --spp 16 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_ml2_1m bash tools/ab.sh "base|" "ml2|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_ml2.so"
