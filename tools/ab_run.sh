cd /root/repo
export STEPS=5 REPEAT=2
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_knot3 bash tools/ab.sh "base|" "gb640|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_gb640.so" "gb640np|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_gb640np.so" && \
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_air3 bash tools/ab.sh "base|" "gb640|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_gb640.so" "gb640np|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_gb640np.so" && \
SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_gb640.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 -k "surface_mesh or airplane" > gpurun_out/ab_air3/parity_gb640.txt 2>&1; tail -3 gpurun_out/ab_air3/parity_gb640.txt
