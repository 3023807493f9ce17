# round 4 call k: launch-claim contention: the tail window (SRT_TAIL_CLAIMS) and the batches per claim (SRT_CLAIM builds)
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04k
F=simple-ray-tracer_amd
C2="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4"
TAG=r04k/c2 REPEAT=1 BENCH_ARGS="$C2" bash tools/ab.sh "c4t16|" "c4t1|SRT_TAIL_CLAIMS=1" "c4t0|SRT_TAIL_CLAIMS=0" \
  "c8t16|SRT_LIB_PATH=$F/libsrt_c8.so" "c8t1|SRT_LIB_PATH=$F/libsrt_c8.so SRT_TAIL_CLAIMS=1" "c8t0|SRT_LIB_PATH=$F/libsrt_c8.so SRT_TAIL_CLAIMS=0" \
  "c16t1|SRT_LIB_PATH=$F/libsrt_c16.so SRT_TAIL_CLAIMS=1" "c16t0|SRT_LIB_PATH=$F/libsrt_c16.so SRT_TAIL_CLAIMS=0" || exit 1
TAG=r04k/rubik REPEAT=1 bash tools/ab.sh "c4t16|" "c4t8|SRT_TAIL_CLAIMS=8" "c8t8|SRT_LIB_PATH=$F/libsrt_c8.so SRT_TAIL_CLAIMS=8" "c8t4|SRT_LIB_PATH=$F/libsrt_c8.so SRT_TAIL_CLAIMS=4" || exit 1
TAG=r04k/torus REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene torusknot --spp 64" bash tools/ab.sh "c4t16|" "c4t4|SRT_TAIL_CLAIMS=4" "c8t8|SRT_LIB_PATH=$F/libsrt_c8.so SRT_TAIL_CLAIMS=8" || exit 1
