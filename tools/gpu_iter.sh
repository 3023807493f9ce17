#!/bin/bash
# development iteration: parity probe + bench (no CPU baseline)
cd /root/repo && export TMPDIR=/tmp
TAG=${TAG:-iter}
mkdir -p gpurun_out/$TAG
timeout -k 10 200 python tools/quick_parity.py > gpurun_out/$TAG/parity.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/$TAG/bench.log 2> gpurun_out/$TAG/bench.err
rc=$?
cat gpurun_out/$TAG/parity.log gpurun_out/$TAG/bench.log
exit $rc
