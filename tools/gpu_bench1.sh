#!/bin/bash
# first bench + kernel-trace profile
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.log 2> gpurun_out/bench1.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
echo "exit $?"
