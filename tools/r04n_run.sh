# round 4 call n: cheap-tile tail claims (SRT_CHEAP_CLAIMS) and the sphere launch's 8-batch claims / tail 1
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04n
F=simple-ray-tracer_amd
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r04n/parity.txt 2>&1 || { tail -20 gpurun_out/r04n/parity.txt; exit 1; }
tail -2 gpurun_out/r04n/parity.txt
NC="nocheap|SRT_LIB_PATH=$F/libsrt_nocheap.so"
TAG=r04n/torus REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene torusknot --spp 64" bash tools/ab.sh "cheap|" "$NC" || exit 1
TAG=r04n/g1m REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --synthetic-tris 1000000 --spp 16" bash tools/ab.sh "cheap|" "$NC" || exit 1
TAG=r04n/s300k REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --synthetic-tris 300000 --spp 16" bash tools/ab.sh "cheap|" "$NC" || exit 1
TAG=r04n/rubik REPEAT=2 bash tools/ab.sh "cheap|" "$NC" || exit 1
TAG=r04n/c2 REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "c8t1|" "c8t16|SRT_TAIL_CLAIMS=16" "c8t0|SRT_TAIL_CLAIMS=0" || exit 1
