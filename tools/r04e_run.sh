# round 4 call e: sphere_kernel with the shadow ray traced in the shading pass that set it up
# (SRT_SPH_SHADOW_NOW): sphere parity, then A/B against the build without it on C2 and C1-size frames
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04e gpurun_out/r04e2
timeout -k 10 400 python -u -m pytest "tests/test_gpu_parity.py::test_spheres_parity" tests/test_gpu_configs.py::test_c1_spheres_256_1spp_full_frame tests/test_gpu_configs.py::test_c2_spheres_1024_64spp_depth4 tests/test_gpu_health.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04e/parity.log 2>&1
rc=$?; echo parity_rc=$rc; tail -3 gpurun_out/r04e/parity.log; [ $rc -ne 0 ] && exit $rc
F=simple-ray-tracer_amd
TAG=r04e2/ab_c2 REPEAT=3 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "ss2|" "ss1|SRT_LIB_PATH=$F/libsrt_ss1.so" "ss0|SRT_LIB_PATH=$F/libsrt_ss0.so" || exit 1
TAG=r04e2/ab_c1 REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 256 --height 256 --spp 1" bash tools/ab.sh "ss2|" "ss0|SRT_LIB_PATH=$F/libsrt_ss0.so" || exit 1
