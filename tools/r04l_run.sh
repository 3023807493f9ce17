# round 4 call l: the tail window and claim size for the global-scene instances (torus knot, 1 M soup, C5)
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04l
F=simple-ray-tracer_amd
TAG=r04l/torus REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene torusknot --spp 64" bash tools/ab.sh "t16|" "t8|SRT_TAIL_CLAIMS=8" "t4|SRT_TAIL_CLAIMS=4" "t2|SRT_TAIL_CLAIMS=2" "t1|SRT_TAIL_CLAIMS=1" "t0|SRT_TAIL_CLAIMS=0" "c8t2|SRT_LIB_PATH=$F/libsrt_c8.so SRT_TAIL_CLAIMS=2" "c8t1|SRT_LIB_PATH=$F/libsrt_c8.so SRT_TAIL_CLAIMS=1" || exit 1
TAG=r04l/g1m REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --synthetic-tris 1000000 --spp 16" bash tools/ab.sh "t16|" "t4|SRT_TAIL_CLAIMS=4" "t2|SRT_TAIL_CLAIMS=2" "t1|SRT_TAIL_CLAIMS=1" "c8t2|SRT_LIB_PATH=$F/libsrt_c8.so SRT_TAIL_CLAIMS=2" || exit 1
TAG=r04l/torus2 REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene torusknot --spp 64" bash tools/ab.sh "t16|" "t4|SRT_TAIL_CLAIMS=4" "t2|SRT_TAIL_CLAIMS=2" "t1|SRT_TAIL_CLAIMS=1" || exit 1
TAG=r04l/c5 REPEAT=1 RUN_TIMEOUT=400 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --width 4096 --height 4096 --spp 16" STEPS=1 bash tools/ab.sh "t16|" "t4|SRT_TAIL_CLAIMS=4" "t1|SRT_TAIL_CLAIMS=1" || exit 1
