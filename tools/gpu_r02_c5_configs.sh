cd /root/repo && O=gpurun_out/r02/c5 bash tools/pmc_c5.sh && bash tools/configs.sh
