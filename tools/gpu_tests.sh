#!/bin/bash
# GPU parity suite + smoke on the box (one process for the tests).
cd /root/repo && export TMPDIR=/tmp
mkdir -p gpurun_out/tests
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/tests/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/tests/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/tests/smoke.log 2>&1; rc=$?
cat gpurun_out/tests/smoke.log; exit $rc
