# round 4 call d: A/B of the fast exact division (SRT_FAST_DIV) and streaming sample stores (SRT_NT_SAMPLES)
# builds against the default, on the metric workload, C2 and the surface-mesh leg; parity of the
# fast-division build on a subset of the GPU suite first
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04d
SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_fd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py::test_c1_spheres_256_1spp_full_frame tests/test_gpu_configs.py::test_c2_spheres_1024_64spp_depth4 -x -q --timeout 300 --timeout-method thread > gpurun_out/r04d/fd_parity.log 2>&1
echo fd_parity_rc=$?; tail -3 gpurun_out/r04d/fd_parity.log
F=simple-ray-tracer_amd
TAG=r04d/ab_rubik REPEAT=2 bash tools/ab.sh "base|" "fd|SRT_LIB_PATH=$F/libsrt_fd.so" "nt|SRT_LIB_PATH=$F/libsrt_nt.so" || exit 1
TAG=r04d/ab_c2 REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "base|" "fd|SRT_LIB_PATH=$F/libsrt_fd.so" "nt|SRT_LIB_PATH=$F/libsrt_nt.so" || exit 1
TAG=r04d/ab_torus REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene torusknot --spp 64" bash tools/ab.sh "base|" "fd|SRT_LIB_PATH=$F/libsrt_fd.so" "nt|SRT_LIB_PATH=$F/libsrt_nt.so" || exit 1
