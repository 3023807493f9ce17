# (SRT_TOP_BFS, SRT_TOP_SHIFT and -DSRT_TOP_PAD were an experiment build, removed after these runs: results in
# profiles/r06_experiments/top_region_bfs.txt and DESIGN.md section 5)
# Round 6 (late): a deeper LDS top region for the 5-wave fused instance -- levels laid out breadth-first and
# cut at the block's LDS share (SRT_TOP_BFS=1), with padded (product) or 64-B (libsrt_t0.so, -DSRT_TOP_PAD=0)
# pair blocks.  Region sizes, a parity subset under each arm, then tools/ab.sh on the two C3-regime legs.
cd /root/repo && export TMPDIR=/tmp
T0=SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_t0.so
for arm in "base|" "bfs|SRT_TOP_BFS=1" "t0|$T0" "t0bfs|$T0 SRT_TOP_BFS=1"; do
  n=${arm%%|*}; e=${arm#*|}
  for s in torusknot airplane_knot synthetic; do
    echo -n "$n: "; env $e timeout -k 10 120 python tools/probes/top_region.py $s || exit 1
  done
done
for arm in "bfs|SRT_TOP_BFS=1" "t0bfs|$T0 SRT_TOP_BFS=1"; do
  env ${arm#*|} timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "top_levels or surface_mesh_global or synthetic_mesh_global or coincident or node_layouts_global or global_schedule or lds_and_global" \
    > gpurun_out/topbfs_parity_${arm%%|*}.txt 2>&1 || { tail -30 gpurun_out/topbfs_parity_${arm%%|*}.txt; exit 1; }
  tail -2 gpurun_out/topbfs_parity_${arm%%|*}.txt
done
export STEPS=5 REPEAT=2
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_topbfs_air \
  bash tools/ab.sh "base|" "bfs|SRT_TOP_BFS=1" "t0bfs|$T0 SRT_TOP_BFS=1" && \
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_topbfs_knot \
  bash tools/ab.sh "base|" "bfs|SRT_TOP_BFS=1" "t0bfs|$T0 SRT_TOP_BFS=1"
