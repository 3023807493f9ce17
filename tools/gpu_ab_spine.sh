cd /root/repo
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/spine_tests.log 2>&1; echo tests rc $?; tail -3 gpurun_out/spine_tests.log
RUNS_FILE=tools/runs_spine.txt TAG=spine bash tools/ab_env.sh && \
RUNS_FILE=tools/runs_spine.txt TAG=spine_c5 STEPS=1 BENCH_ARGS="--scene synthetic --width 4096 --height 4096 --spp 16 --no-global-leg" bash tools/ab_env.sh
