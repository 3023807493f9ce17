# Round 6 (late): the fused global-scene instance's sub-steps per traversal iteration re-swept on the C3-regime
# legs (builds -DSRT_GLOBAL_FUSED=6/10/12; the product's is 8, tuned in round 4 on the inward knot).
cd /root/repo && export TMPDIR=/tmp STEPS=5 REPEAT=2
L=simple-ray-tracer_amd
A="f6|SRT_LIB_PATH=$L/libsrt_f6.so"; B="f10|SRT_LIB_PATH=$L/libsrt_f10.so"; C="f12|SRT_LIB_PATH=$L/libsrt_f12.so"
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_fused_air \
  bash tools/ab.sh "base|" "$A" "$B" "$C" && \
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_fused_knot \
  bash tools/ab.sh "base|" "$A" "$B" "$C"
