#!/bin/bash
# Round-2 closing run on the three-triangle LDS kernel: GPU suite + smoke, round profile (bench line, kernel
# trace, PMC passes), C2/C4 PMC passes, the BASELINE configs.
cd /root/repo && export TMPDIR=/tmp
bash tools/gpu_tests.sh && \
ROUND=r02c bash tools/profile_round.sh && \
bash tools/pmc_configs.sh && \
bash tools/configs.sh
