# Round 6 (late): LDS mode reads the stack's top entry with each sub-step's node/triangle reads, so a lane that
# (-DSRT_POP_PREFETCH was an experiment build, removed after this run: profiles/r06_experiments/pop_prefetch.txt)
# ends the sub-step with nothing current pops without a second LDS round trip (-DSRT_POP_PREFETCH=1 build).
cd /root/repo && export TMPDIR=/tmp
V=SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_pp.so
env $V timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "rubik_parity or coincident or moved_camera_parity or lds_budget or pathological or ghost or two_models or lights" \
  > gpurun_out/pp_parity.txt 2>&1 || { tail -30 gpurun_out/pp_parity.txt; exit 1; }
tail -1 gpurun_out/pp_parity.txt
export STEPS=5 REPEAT=3
TAG=ab_pp_metric bash tools/ab.sh "base|" "pp|$V"
