#!/bin/bash
# The first half of tools/gpu_round_close.sh, for a GPU call of its own (each call is capped at 20 min):
# every workload's profile passes (tools/gpu_profiles.sh + tools/pmc_configs.sh) and profiles/counters.json
# rebuilt from them on the box (copied to gpurun_out/$R/counters.json to bring it back).  The second
# half is tools/gpu_close.sh (GPU suite + smoke, the bench line with its roofs, the config lines).
cd /root/repo && export TMPDIR=/tmp
R=${ROUND:?set ROUND}
ROUND=$R bash tools/gpu_profiles.sh || exit 1
timeout -k 10 900 bash tools/pmc_configs.sh > gpurun_out/${R}_pmc_configs.log 2>&1 || { echo "pmc_configs failed"; exit 1; }
python3 tools/pmc_roofline.py gpurun_out/$R --tag $R && \
python3 tools/pmc_roofline.py gpurun_out/${R}_c5 --workload synthetic10000000_4096x4096_16spp --il --tag $R && \
python3 tools/pmc_roofline.py gpurun_out/pmc_c2 --workload spheres_1024x1024_64spp_depth4 --sum --tag $R && \
python3 tools/pmc_roofline.py gpurun_out/pmc_c4 --workload rubik_4096x4096_1024spp_depth8 --sum --tag $R || { echo "pmc_roofline failed"; exit 1; }
cp profiles/counters.json gpurun_out/$R/counters.json
echo "round profiles done"
