# round 4 call o: sharded batch counters (kBatchHeads, one per XCD group) against one counter (SRT_BATCH_HEADS=1)
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04o
F=simple-ray-tracer_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r04o/parity.txt 2>&1 || { tail -20 gpurun_out/r04o/parity.txt; exit 1; }
tail -1 gpurun_out/r04o/parity.txt
H1="h1|SRT_LIB_PATH=$F/libsrt_h1.so"
TAG=r04o/c2 REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "h8|" "$H1" "h8t16|SRT_TAIL_CLAIMS=16" "h8c4|SRT_LIB_PATH=$F/libsrt_h8c4.so" "h8c4t16|SRT_LIB_PATH=$F/libsrt_h8c4.so SRT_TAIL_CLAIMS=16" || exit 1
TAG=r04o/torus REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene torusknot --spp 64" bash tools/ab.sh "h8|" "$H1" "h8t4|SRT_TAIL_CLAIMS=4" || exit 1
TAG=r04o/g1m REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --synthetic-tris 1000000 --spp 16" bash tools/ab.sh "h8|" "$H1" || exit 1
TAG=r04o/s300k REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --synthetic-tris 300000 --spp 16" bash tools/ab.sh "h8|" "$H1" || exit 1
TAG=r04o/rubik REPEAT=2 bash tools/ab.sh "h8|" "$H1" || exit 1
