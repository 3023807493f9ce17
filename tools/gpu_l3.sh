#!/bin/bash
# A/B of three-triangle leaf steps in LDS mode (SRT_LEAF_TRIS_LDS=3; ${RUNS:-tools/runs/l3.txt}), after a parity
# probe of the l3 build on the LDS-mode tests.
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/l3
SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_l3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
  --timeout 200 --timeout-method thread -k "rubik or sphere or lds or budget or spp" > gpurun_out/l3/tests.log 2>&1
rc=$?; tail -2 gpurun_out/l3/tests.log; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-l3} RUNS_FILE=${RUNS:-tools/runs/l3.txt} bash tools/ab_env.sh
