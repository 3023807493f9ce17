#!/bin/bash
# GPU suite + smoke (tools/gpu_tests.sh), then C5 at higher global-mode early-break thresholds.
cd /root/repo && export TMPDIR=/tmp
bash tools/gpu_tests.sh && \
TAG=gfrac_c5b STEPS=1 RUNS_FILE=tools/runs/gfrac_c5b.txt \
  BENCH_ARGS="--scene synthetic --width 4096 --height 4096 --spp 16 --no-global-leg --no-surface-leg" bash tools/ab_env.sh
