# round 4 call h: the tile-cost record's tile index kept in a register (SRT_TILE_IDX_REG) vs the division
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04h
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04h/parity.log 2>&1
rc=$?; echo parity_rc=$rc; tail -2 gpurun_out/r04h/parity.log; [ $rc -ne 0 ] && exit $rc
F=simple-ray-tracer_amd
TAG=r04h/ab_rubik REPEAT=2 bash tools/ab.sh "ti|" "ti0|SRT_LIB_PATH=$F/libsrt_ti0.so" || exit 1
TAG=r04h/ab_torus REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene torusknot --spp 64" bash tools/ab.sh "ti|" "ti0|SRT_LIB_PATH=$F/libsrt_ti0.so" || exit 1
TAG=r04h/ab_1m REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --synthetic-tris 1000000 --spp 16" bash tools/ab.sh "ti|" "ti0|SRT_LIB_PATH=$F/libsrt_ti0.so" || exit 1
TAG=r04h/ab_c2 REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "ti|" "ti0|SRT_LIB_PATH=$F/libsrt_ti0.so" || exit 1
