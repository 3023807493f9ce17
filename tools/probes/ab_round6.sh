# Round 6's last A/B runs (tools/ab.sh): the fused global instance's batches strip by strip (-DSRT_STRIPS=K builds)
cd /root/repo
export STEPS=5 REPEAT=2
L=simple-ray-tracer_amd
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_st_air bash tools/ab.sh "base|" "st4|SRT_LIB_PATH=$L/libsrt_st4.so" "st8|SRT_LIB_PATH=$L/libsrt_st8.so" "st16|SRT_LIB_PATH=$L/libsrt_st16.so" && \
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_st_knot bash tools/ab.sh "base|" "st4|SRT_LIB_PATH=$L/libsrt_st4.so" "st8|SRT_LIB_PATH=$L/libsrt_st8.so" "st16|SRT_LIB_PATH=$L/libsrt_st16.so" && \
SRT_LIB_PATH=$L/libsrt_st8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 -k "surface_mesh or airplane" > gpurun_out/ab_st_air/parity_st8.txt 2>&1; tail -2 gpurun_out/ab_st_air/parity_st8.txt
