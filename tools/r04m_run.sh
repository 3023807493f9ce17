# round 4 call m: the tail window on other scenes of the 5-wave fused instance (soups under 48 MB), Rubik forced global
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04m
TAG=r04m/s300k REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --synthetic-tris 300000 --spp 16" bash tools/ab.sh "t16|" "t4|SRT_TAIL_CLAIMS=4" "t2|SRT_TAIL_CLAIMS=2" || exit 1
TAG=r04m/s100k REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --synthetic-tris 100000 --spp 16" bash tools/ab.sh "t16|" "t4|SRT_TAIL_CLAIMS=4" "t2|SRT_TAIL_CLAIMS=2" || exit 1
TAG=r04m/rubikg REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --spp 64" bash tools/ab.sh "t16|SRT_FORCE_GLOBAL_SCENE=1" "t4|SRT_FORCE_GLOBAL_SCENE=1 SRT_TAIL_CLAIMS=4" "t2|SRT_FORCE_GLOBAL_SCENE=1 SRT_TAIL_CLAIMS=2" || exit 1
TAG=r04m/torus_c2cmp REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene torusknot --spp 64" bash tools/ab.sh "t16|" "t2|SRT_TAIL_CLAIMS=2" "t3|SRT_TAIL_CLAIMS=3" || exit 1
