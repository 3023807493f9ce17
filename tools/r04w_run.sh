# round 4 call w: the round's close on the final build, then C5's step with and without the pipeline slots
cd /root/repo && export TMPDIR=/tmp
ROUND=r04w bash tools/gpu_round_close.sh || exit 1
TAG=r04w/c5 REPEAT=1 RUN_TIMEOUT=400 STEPS=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --width 4096 --height 4096 --spp 16" bash tools/ab.sh "p3|" "p1|SRT_PIPELINE=1" || exit 1
