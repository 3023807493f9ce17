# Round 6 (late): the device code built without LLVM's SLP vectorizer (-fno-slp-vectorize): it pairs
# independent f32 operations into v_pk_* instructions at the cost of v_mov shuffles and registers (the
# 3-triangle leaf step: 201 VALU with it, 180 without; the metric kernel's spills 28 B -> 0).  A parity subset
# under the variant, then tools/ab.sh on the metric workload, the two C3-regime legs and C2.
cd /root/repo && export TMPDIR=/tmp
V=SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_noslp.so
env $V timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "rubik_parity or spheres_parity or surface_mesh_global or synthetic_mesh_global or coincident or top_levels or sampled_texture_parity or trace_closest" \
  > gpurun_out/noslp_parity.txt 2>&1 || { tail -30 gpurun_out/noslp_parity.txt; exit 1; }
tail -1 gpurun_out/noslp_parity.txt
export STEPS=5 REPEAT=2
TAG=ab_noslp_metric bash tools/ab.sh "base|" "noslp|$V" && \
BENCH_ARGS="--scene airplane_knot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_noslp_air \
  bash tools/ab.sh "base|" "noslp|$V" && \
BENCH_ARGS="--scene torusknot --spp 64 --no-global-leg --no-surface-leg --no-airplane-leg" TAG=ab_noslp_knot \
  bash tools/ab.sh "base|" "noslp|$V" && \
BENCH_ARGS="--no-global-leg --no-surface-leg --no-airplane-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" \
  STEPS=20 TAG=ab_noslp_c2 bash tools/ab.sh "base|" "noslp|$V"
