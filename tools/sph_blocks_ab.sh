cd /root/repo && export TMPDIR=/tmp
H="head|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_head.so"
BENCH_ARGS="--scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4 --no-global-leg --no-surface-leg" TAG=sp_sph2 REPEAT=3 STEPS=5 bash tools/ab.sh "$H" "b4|SRT_SPHERE_BLOCKS=4" "b5|SRT_SPHERE_BLOCKS=5" "b3|SRT_SPHERE_BLOCKS=3" "b6|SRT_SPHERE_BLOCKS=6"
