#!/bin/bash
# Round-2 closing profile on the padded-LDS-node kernel: bench line, rocprofv3 kernel trace, PMC passes
# (tools/profile_round.sh), then an early-break threshold re-sweep on the metric workload.
cd /root/repo && export TMPDIR=/tmp
ROUND=r02b bash tools/profile_round.sh && \
TAG=frac_r2 RUNS_FILE=tools/runs/frac_r2.txt bash tools/ab_env.sh
