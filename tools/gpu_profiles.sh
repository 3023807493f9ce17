#!/bin/bash
# The round's closing profiles in one GPU call: bench line + kernel trace + PMC passes of the metric
# workload and both legs (tools/profile_round.sh), then C5's passes (tools/pmc_c5.sh).  C2/C4 passes and
# the config lines: tools/pmc_configs.sh and tools/configs.sh (a second call).
cd /root/repo && export TMPDIR=/tmp
R=${ROUND:?set ROUND}
ROUND=$R bash tools/profile_round.sh > gpurun_out/${R}_profile.log 2>&1 || { echo "profile_round failed"; tail -5 gpurun_out/${R}_profile.log; exit 1; }
O=gpurun_out/${R}_c5 bash tools/pmc_c5.sh > gpurun_out/${R}_c5.log 2>&1 || { echo "pmc_c5 failed"; tail -5 gpurun_out/${R}_c5.log; exit 1; }
echo "profiles done"
