#!/bin/bash
# PMC passes of the C5 workload (synthetic 10M triangles, 4096^2 @16 spp, one timed launch) for
# profiles/counters.json (tools/pmc_roofline.py <dir> --workload synthetic10000000_4096x4096_16spp).
cd /root/repo && export TMPDIR=/tmp
# (PMC passes run their launches in series, SRT_PIPELINE_OVERLAP=0: the same kernels and work; an overlapped
# launch's counter window would also hold its wait for the CUs another launch holds, doubling its cycle counters)
O=${O:-gpurun_out/c5pmc}; mkdir -p $O
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-global-leg --no-surface-leg --no-airplane-leg --scene synthetic --width 4096 --height 4096 --spp 16"
SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
  SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o run -- \
  $B > $O/pmc_sq.log 2>&1 && \
SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 && \
SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 && \
SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_tcc -o run -- $B > $O/pmc_tcc.log 2>&1
rc=$?; echo "pmc exit $rc"; exit $rc
