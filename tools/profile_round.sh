#!/bin/bash
# Round profile: bench line + rocprofv3 kernel trace + PMC passes (one counter group per run) for
# profiles/counters.json (tools/pmc_roofline.py): the roofs bench.py reports.
cd /root/repo && export TMPDIR=/tmp
R=${ROUND:-r02}; O=gpurun_out/$R; mkdir -p $O
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
  SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o run -- \
  $B > $O/pmc_sq.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1
rc=$?; echo "profile exit $rc"; cat $O/bench.json; exit $rc
