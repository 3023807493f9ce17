#!/bin/bash
# GPU parity suite + smoke on the box (one process for the tests).
cd /root/repo && export TMPDIR=/tmp
mkdir -p gpurun_out/tests
# a heartbeat line a minute: the at-size config tests run minutes without a line of pytest output
( while sleep 60; do date +"%T tests running" >> gpurun_out/tests/heartbeat.log; done ) &
hb=$!
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=12 \
  > gpurun_out/tests/gpu_tests.log 2>&1
rc=$?
kill $hb
tail -30 gpurun_out/tests/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/tests/smoke.log 2>&1; rc=$?
cat gpurun_out/tests/smoke.log; exit $rc
