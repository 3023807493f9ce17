# round 4 call p: sphere_kernel blocks per CU once the claim counter no longer bounds C2
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04p
TAG=r04p/c2 REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "b3|" "b2|SRT_SPHERE_BLOCKS=2" "b4|SRT_SPHERE_BLOCKS=4" "b5|SRT_SPHERE_BLOCKS=5" || exit 1
# the N-GPU rank share of the metric by row-band height (an 8x8 tile of a 2-row-band share spans 64 image rows at N = 8)
for b in 2 8 16; do timeout -k 10 300 python tools/tail_sweep.py rubik 256 $b 16 2>/dev/null | tee -a gpurun_out/r04p/bands.txt || exit 1; done
