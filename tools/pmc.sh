#!/bin/bash
# PMC passes (counters only with --kernel-trace-free --pmc; one group per pass)
cd /root/repo && export TMPDIR=/tmp
SPP=${SPP:-32}
TAG=${TAG:-pmc}
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/$TAG/$name -o run -- \
    python bench.py --steps 1 --warmup 0 --spp $SPP --no-cpu-baseline $BENCH_ARGS > gpurun_out/$TAG/$name.log 2>&1
}
mkdir -p gpurun_out/$TAG
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && \
run p2 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS && \
run p3 FETCH_SIZE && \
run p4 WRITE_SIZE && \
run p5 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum && \
run p6 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32
echo "pmc exit $?"
