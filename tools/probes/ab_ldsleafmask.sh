# Round 6 (late): LDS mode reads only a leaf's remaining triangles in each 3-triangle leaf step (records past
# (-DSRT_LDS_LEAF_MASK was an experiment build, removed after this run: profiles/r06_experiments/lds_leaf_mask.txt)
# the leaf are zero constants: -DSRT_LDS_LEAF_MASK=1 build), against the product: parity subset, then the
# metric workload and C4.
cd /root/repo && export TMPDIR=/tmp
V=SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_lm.so
env $V timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "rubik_parity or coincident or moved_camera_parity or lds_budget or pathological or ghost or two_models or lights" \
  > gpurun_out/lm_parity.txt 2>&1 || { tail -30 gpurun_out/lm_parity.txt; exit 1; }
tail -1 gpurun_out/lm_parity.txt
export STEPS=5 REPEAT=3
TAG=ab_lm_metric bash tools/ab.sh "base|" "lm|$V"
