#!/bin/bash
# GPU parity suite on the default build, then A/B of the camera-noise prefetch (tools/runs/nzpf.txt).
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/nzpf
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/nzpf/tests.log 2>&1
rc=$?; tail -3 gpurun_out/nzpf/tests.log; [ $rc -ne 0 ] && exit $rc
TAG=nzpf RUNS_FILE=tools/runs/nzpf.txt bash tools/ab_env.sh
