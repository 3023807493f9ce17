# round 4 call c: the whole GPU suite + smoke on the reverted build, then the C2 occupancy counter study
cd /root/repo && export TMPDIR=/tmp
bash tools/gpu_tests.sh > gpurun_out/r04c_tests.log 2>&1; rc=$?; tail -6 gpurun_out/r04c_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/c2_study.sh > gpurun_out/r04c_c2.log 2>&1; rc=$?; cat gpurun_out/r04c_c2.log; [ $rc -ne 0 ] && exit $rc
python3 tools/c2_study.py gpurun_out/c2s --out gpurun_out/r04c_c2_study.json
bash tools/pmc_study.sh torus "--scene torusknot --spp 64" "gw5|" "gw4|SRT_GLOBAL_WAVES_MODE=4" > gpurun_out/r04c_torus.log 2>&1; rc=$?; cat gpurun_out/r04c_torus.log; [ $rc -ne 0 ] && exit $rc
python3 tools/c2_study.py gpurun_out/torus --kernel "void srt::sample_kernel<false" --out gpurun_out/r04c_torus_study.json
