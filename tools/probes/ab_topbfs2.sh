# (SRT_TOP_BFS, SRT_TOP_SHIFT and -DSRT_TOP_PAD were an experiment build, removed after these runs: results in
# profiles/r06_experiments/top_region_bfs.txt and DESIGN.md section 5)
# Round 6 (late), after the LDS-unit fix (GlobalBlockLds: 32,000 B per block at 5 blocks per CU): the
# breadth-first region cut at the corrected share, padded (product stride) and 64-B (libsrt_t0.so) blocks.
cd /root/repo && export TMPDIR=/tmp
T0=SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_t0.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "occupancy or top_levels or global_schedule" > gpurun_out/topbfs2_tests.txt 2>&1 || { tail -30 gpurun_out/topbfs2_tests.txt; exit 1; }
tail -1 gpurun_out/topbfs2_tests.txt
for arm in "base|" "bfs|SRT_TOP_BFS=1" "t0bfs|$T0 SRT_TOP_BFS=1"; do
  echo -n "${arm%%|*}: "; env ${arm#*|} timeout -k 10 120 python tools/probes/top_region.py airplane_knot || exit 1
done
export STEPS=5 REPEAT=2
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_topbfs2_air \
  bash tools/ab.sh "base|" "bfs|SRT_TOP_BFS=1" "t0bfs|$T0 SRT_TOP_BFS=1" && \
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_topbfs2_knot \
  bash tools/ab.sh "base|" "bfs|SRT_TOP_BFS=1" "t0bfs|$T0 SRT_TOP_BFS=1"
