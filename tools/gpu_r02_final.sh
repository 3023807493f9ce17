#!/bin/bash
# Round-2 closing measurements: C5 PMC passes, the other BASELINE configs, then the bench line with the
# committed counters (run after tools/profile_round.sh + tools/pmc_roofline.py).
cd /root/repo && export TMPDIR=/tmp
O=gpurun_out/r02/c5 bash tools/pmc_c5.sh && bash tools/configs.sh && \
timeout -k 10 600 python bench.py > gpurun_out/r02/bench_final.json 2> gpurun_out/r02/bench_final.err
rc=$?; echo "final exit $rc"; exit $rc
