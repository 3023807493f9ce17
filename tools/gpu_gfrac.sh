#!/bin/bash
# Early-break threshold sweep for global-scene mode (SRT_TRAV_FRAC16_GLOBAL): the bench legs, then C5.
cd /root/repo && export TMPDIR=/tmp
TAG=gfrac RUNS_FILE=tools/runs/gfrac.txt bash tools/ab_env.sh && \
TAG=gfrac_c5 STEPS=1 RUNS_FILE=tools/runs/gfrac_c5.txt \
  BENCH_ARGS="--scene synthetic --width 4096 --height 4096 --spp 16 --no-global-leg --no-surface-leg" bash tools/ab_env.sh
