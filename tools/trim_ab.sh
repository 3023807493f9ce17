cd /root/repo && export TMPDIR=/tmp
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg" TAG=trim_torus REPEAT=3 bash tools/ab.sh "base|" "sr|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_sr.so" "nt|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_nt.so" "both|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_both.so" || exit 1
BENCH_ARGS="--no-global-leg --no-surface-leg" TAG=trim_rubik REPEAT=2 bash tools/ab.sh "base|" "sr|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_sr.so" "both|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_both.so"
