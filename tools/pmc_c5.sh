#!/bin/bash
# PMC passes on the C5 synthetic scene (global-scene mode), reduced frame
cd /root/repo && export TMPDIR=/tmp
TAG=${TAG:-pmc_c5}; A="--scene synthetic --width 2048 --height 2048 --spp 4 --steps 1 --warmup 0 --no-cpu-baseline"
run() { local name=$1; shift
  timeout -k 10 600 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/$TAG/$name -o run -- \
    python bench.py $A > gpurun_out/$TAG/$name.log 2>&1; }
mkdir -p gpurun_out/$TAG
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && \
run p2 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR && \
run p3 FETCH_SIZE && run p4 WRITE_SIZE && \
run p5 TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum && \
run p6 TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum
echo "pmc exit $?"
