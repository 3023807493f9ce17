#!/bin/bash
# The bench line (defaults, CPU baseline included) and the BASELINE configs on the committed r02c counters.
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r02c
timeout -k 10 600 python bench.py > gpurun_out/r02c/bench_final.json 2> gpurun_out/r02c/bench_final.err && \
bash tools/configs.sh
rc=$?; cat gpurun_out/r02c/bench_final.json; exit $rc
