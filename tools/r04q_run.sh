# round 4 call q: sphere_kernel at 5 blocks per CU (default now) vs a 6-wave register bound (80 VGPRs, 12 spilled)
cd /root/repo && export TMPDIR=/tmp; mkdir -p gpurun_out/r04q
F=simple-ray-tracer_amd
TAG=r04q/c2 REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "b5|" "b4|SRT_SPHERE_BLOCKS=4" "w6b6|SRT_LIB_PATH=$F/libsrt_s6.so SRT_SPHERE_BLOCKS=6" || exit 1
