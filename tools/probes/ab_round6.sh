# Round 6's last A/B runs (tools/ab.sh): node and triangle layouts on the C3-regime legs
cd /root/repo
export STEPS=5 REPEAT=2
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_lay_air bash tools/ab.sh "base|" "na1|SRT_NODE_ALIGN=1" "ta0|SRT_TRI_ALIGN=0" && \
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_lay_knot bash tools/ab.sh "base|" "na1|SRT_NODE_ALIGN=1" "ta0|SRT_TRI_ALIGN=0"
