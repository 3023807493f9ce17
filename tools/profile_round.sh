#!/bin/bash
# Round profile: bench line + rocprofv3 kernel trace + PMC passes (one counter group per run) for
# profiles/counters.json (tools/pmc_roofline.py): the roofs bench.py reports.
cd /root/repo && export TMPDIR=/tmp
R=${ROUND:-r02}; O=gpurun_out/$R; mkdir -p $O
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
# The PMC passes time their launch in series (SRT_PIPELINE_OVERLAP=0: the same kernels and work; an
# overlapped launch's counter window would also hold its wait for the CUs another launch holds, which
# doubles its cycle counters); the bench line and the kernel trace keep the default (overlapped).
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python bench.py --steps 10 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 && \
T=$(find $O/trace -name "*kernel_trace.csv" | head -1) && \
python3 tools/trace_intervals.py $T "sample_kernel<false, true, true, 1024, false, false, 4>" 10 $O/trace.log > $O/intervals.json && \
SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
  SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o run -- \
  $B > $O/pmc_sq.log 2>&1 && \
SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 \
  SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/pmc_sq2 -o run -- \
  $B > $O/pmc_sq2.log 2>&1 && \
SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 && \
SRT_PIPELINE_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1
rc=$?; echo "profile exit $rc"; cat $O/bench.json; exit $rc
