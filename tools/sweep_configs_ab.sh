cd /root/repo && export TMPDIR=/tmp
TAG=sw4 SWEEP_FILE=tools/runs/sweep_r1e.txt bash tools/sweep.sh && \
TAG=sw4s SWEEP_FILE=tools/runs/sweep_r1e.txt BENCH_ARGS="--scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/sweep.sh && \
TAG=sw4g SWEEP_FILE=tools/runs/sweep_r1e.txt BENCH_ARGS="--scene synthetic --synthetic-tris 1000000 --spp 16" bash tools/sweep.sh && \
TAG=sw4r SWEEP_FILE=tools/runs/sweep_r1e.txt BENCH_ARGS="--width 4096 --height 4096 --spp 128 --max-depth 8" bash tools/sweep.sh
