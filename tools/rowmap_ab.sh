#!/bin/bash
# Row-band table in the refill (kp.row_map) vs the band arithmetic (libsrt_head.so): multi-rank parity, then A/B.
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wavefront.py -k "band or tiling or rank" -x -q --timeout 200 --timeout-method thread > gpurun_out/rowmap_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/rowmap_tests.log; exit 1; }
tail -2 gpurun_out/rowmap_tests.log
BENCH_ARGS="--no-global-leg --no-surface-leg" TAG=rm_rubik REPEAT=3 bash tools/ab.sh "head|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_head.so" "rowmap|" || exit 1
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg" TAG=rm_torus REPEAT=3 bash tools/ab.sh "head|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_head.so" "rowmap|"
