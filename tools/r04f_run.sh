# round 4 call f: sphere_kernel draws prefetched one iteration ahead (SRT_SPH_PREFETCH): parity, A/B
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04f
timeout -k 10 400 python -u -m pytest "tests/test_gpu_parity.py::test_spheres_parity" tests/test_gpu_configs.py::test_c1_spheres_256_1spp_full_frame tests/test_gpu_configs.py::test_c2_spheres_1024_64spp_depth4 tests/test_gpu_health.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04f/parity.log 2>&1
rc=$?; echo parity_rc=$rc; tail -3 gpurun_out/r04f/parity.log; [ $rc -ne 0 ] && exit $rc
F=simple-ray-tracer_amd
TAG=r04f/ab_c2 REPEAT=3 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "pf|" "pf0|SRT_LIB_PATH=$F/libsrt_pf0.so" "pf_b4|SRT_SPHERE_BLOCKS=4" || exit 1
TAG=r04f/ab_rubik REPEAT=1 bash tools/ab.sh "pf|" "pf0|SRT_LIB_PATH=$F/libsrt_pf0.so" || exit 1
