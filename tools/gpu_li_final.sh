#!/bin/bash
# A/B of the leaf-first sub-step pattern, then the default bench line (with the CPU baseline) on the
# committed r02b counters.
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r02b
TAG=li RUNS_FILE=tools/runs/li.txt bash tools/ab_env.sh && \
timeout -k 10 600 python bench.py > gpurun_out/r02b/bench_final.json 2> gpurun_out/r02b/bench_final.err
rc=$?; cat gpurun_out/r02b/bench_final.json; exit $rc
