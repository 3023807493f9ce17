#!/bin/bash
# GPU A/B of library builds / env knobs: the GPU suite on the default build, then the metric workload
# with its global-scene leg and C5 (synthetic 10M, 4096^2 @16 spp) for every line of RUNS_FILE
# ("name|ENV=value ..."; SRT_LIB_PATH selects a variant build).  Usage on the box:
#   RUNS_FILE=tools/runs_x.txt bash tools/gpu_ab.sh
cd /root/repo
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
fi
TAG=ab bash tools/ab_env.sh && \
TAG=ab_c5 STEPS=1 BENCH_ARGS="--scene synthetic --width 4096 --height 4096 --spp 16 --no-global-leg" bash tools/ab_env.sh
