# Round 6 (late): LDS mode's sub-step pattern re-swept on the round-6 kernel (builds
# -DSRT_STEP_PATTERN_LDS='"..."'; the product's is IILILILILIL), metric workload.
cd /root/repo && export TMPDIR=/tmp STEPS=5 REPEAT=2
L=simple-ray-tracer_amd
TAG=ab_lds_pattern bash tools/ab.sh "base|" "p13|SRT_LIB_PATH=$L/libsrt_p13.so" "p9|SRT_LIB_PATH=$L/libsrt_p9.so" \
  "p12a|SRT_LIB_PATH=$L/libsrt_p12a.so" "p12b|SRT_LIB_PATH=$L/libsrt_p12b.so"
