#!/bin/bash
# A/B (RUNS_FILE lines) of the global-scene mode on synthetic meshes of several sizes, 1920x1080 @16 spp.
cd /root/repo
for T in ${SIZES:-300000 3000000}; do
  TAG=ab_t$T STEPS=2 BENCH_ARGS="--scene synthetic --synthetic-tris $T --spp 16 --no-global-leg" bash tools/ab_env.sh || exit 1
done
