#!/bin/bash
cd /root/repo && export TMPDIR=/tmp
mkdir -p gpurun_out/tests
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/tests/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/tests/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/tests/smoke.log 2>&1; rc=$?
cat gpurun_out/tests/smoke.log; exit $rc
