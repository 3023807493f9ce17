#!/bin/bash
# Claim size / tail window on the LDS kernel; "II"-first IL patterns for global-scene mode on C5.
cd /root/repo && export TMPDIR=/tmp
TAG=r2misc RUNS_FILE=tools/runs/r2misc.txt bash tools/ab_env.sh && \
TAG=r2misc_c5 STEPS=1 RUNS_FILE=tools/runs/r2misc_c5.txt \
  BENCH_ARGS="--scene synthetic --width 4096 --height 4096 --spp 16 --no-global-leg --no-surface-leg" bash tools/ab_env.sh
