#!/bin/bash
# Mesh/sphere code split (sphere_kernel): GPU parity suite, then A/B against libsrt_head.so.
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/split_tests.log; exit 1; }
tail -2 gpurun_out/split_tests.log
H="head|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_head.so"
BENCH_ARGS="--no-global-leg --no-surface-leg" TAG=sp_rubik REPEAT=3 bash tools/ab.sh "$H" "split|" || exit 1
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg" TAG=sp_torus REPEAT=3 bash tools/ab.sh "$H" "split|" || exit 1
BENCH_ARGS="--scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4 --no-global-leg --no-surface-leg" TAG=sp_sph REPEAT=3 STEPS=5 bash tools/ab.sh "$H" "split|" || exit 1
BENCH_ARGS="--scene synthetic --synthetic-tris 1000000 --spp 16 --no-global-leg --no-surface-leg" TAG=sp_soup REPEAT=2 bash tools/ab.sh "$H" "split|"
