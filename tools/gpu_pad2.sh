#!/bin/bash
# A/B of the padded LDS node layout (base: SRT_NODE_PAD=0) + the phase split of the LDS kernel.
cd /root/repo && export TMPDIR=/tmp
TAG=pad2 RUNS_FILE=tools/runs/pad.txt bash tools/ab_env.sh || exit 1
SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_phase.so timeout -k 10 200 python tools/phase_timing.py 32 > gpurun_out/pad2/phase.txt 2>&1; rc=$?
cat gpurun_out/pad2/phase.txt; exit $rc
