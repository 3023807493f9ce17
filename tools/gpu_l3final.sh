#!/bin/bash
# GPU suite + smoke on the three-triangle / 10-sub-step LDS kernel, A/B against the previous kernel, then
# the BASELINE configs.
cd /root/repo && export TMPDIR=/tmp
bash tools/gpu_tests.sh && \
TAG=l3final RUNS_FILE=tools/runs/l3final.txt bash tools/ab_env.sh && \
bash tools/configs.sh
