# (SRT_TOP_BFS, SRT_TOP_SHIFT and -DSRT_TOP_PAD were an experiment build, removed after these runs: results in
# profiles/r06_experiments/top_region_bfs.txt and DESIGN.md section 5)
# Round 6 (late): why the breadth-first region lost 11% -- its order (no right-spine flags in the region) or
# the 64-B shift of every pair below it against the 128-B lines.  SRT_TOP_SHIFT=k puts k zero pairs (64 B
# each) between the region and the rest; SRT_TOP_BFS=1 SRT_TOP_DEPTH=7 is the breadth-first region at the
# product's size.
cd /root/repo && export TMPDIR=/tmp STEPS=5 REPEAT=2
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_topshift_air \
  bash tools/ab.sh "base|" "s1|SRT_TOP_SHIFT=1" "s2|SRT_TOP_SHIFT=2" "bfs7|SRT_TOP_BFS=1 SRT_TOP_DEPTH=7"
