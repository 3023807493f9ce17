#!/bin/bash
# Memory-counter calibration for the traversal's access patterns (tools/gather_calib.hip): a timing run,
# then one rocprofv3 PMC pass per counter group over the same launches; tools/gather_calib.py joins them.
cd /root/repo && export TMPDIR=/tmp
O=${O:-gpurun_out/calib}; mkdir -p $O
timeout -k 10 120 ./tools/gather_calib 3 > $O/timing.txt 2> $O/timing.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- ./tools/gather_calib 1 \
  > $O/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum \
  --output-format csv -d $O/pmc_req -o run -- ./tools/gather_calib 1 > $O/pmc_req.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_tcc -o run -- \
  ./tools/gather_calib 1 > $O/pmc_tcc.log 2>&1
rc=$?; echo "calib exit $rc"; cat $O/timing.txt; exit $rc
