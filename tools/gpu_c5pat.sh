#!/bin/bash
# GPU suite + smoke with the IIL... global IL pattern, then C5.
cd /root/repo && export TMPDIR=/tmp
bash tools/gpu_tests.sh && \
TAG=c5pat STEPS=1 RUNS_FILE=tools/runs/c5pat.txt \
  BENCH_ARGS="--scene synthetic --width 4096 --height 4096 --spp 16 --no-global-leg --no-surface-leg" bash tools/ab_env.sh
