#!/bin/bash
# PMC passes of the C2 and C4 configs (tools/configs.sh's workloads, one timed step each) for
# profiles/counters.json: python tools/pmc_roofline.py gpurun_out/pmc_c2 --workload spheres_1024x1024_64spp_depth4 --sum
# and gpurun_out/pmc_c4 --workload rubik_4096x4096_1024spp_depth8 --sum.
cd /root/repo && export TMPDIR=/tmp
# (PMC passes run their launches in series, SRT_PIPELINE_OVERLAP=0: the same kernels and work; an overlapped
# launch's counter window would also hold its wait for the CUs another launch holds, doubling its cycle counters)
pass() { local O=$1; shift
  mkdir -p $O
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
    SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o run -- \
    "$@" > $O/pmc_sq.log 2>&1 && \
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- "$@" > $O/pmc_fetch.log 2>&1 && \
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- "$@" > $O/pmc_write.log 2>&1; }
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-global-leg --no-surface-leg --no-airplane-leg"
pass gpurun_out/pmc_c2 $B --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4 && \
pass gpurun_out/pmc_c4 $B --scene rubik --width 4096 --height 4096 --spp 1024 --max-depth 8
rc=$?; echo "pmc exit $rc"; exit $rc
