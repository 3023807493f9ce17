#!/bin/bash
# Vector-memory pipeline study of one workload under several variants: is a global-scene kernel bound by the
# address path (TA: one address per lane of a divergent gather), the data return (TD), the L1/L2 request
# path (TCP), address translation (UTCL1), or by latency alone?  Per variant: bench.py's kernel time and
# one rocprofv3 pass per counter group (at most 2 TA, 2 TD, 4 TCP, 2 GRBM counters a pass; launches in
# series, SRT_PIPELINE_OVERLAP=0).  Reduced by tools/c2_study.py (vmem keys).
#   tools/vmem_study.sh NAME "BENCH ARGS" "var1|ENV=x" ...     -> gpurun_out/NAME/<var>/
cd /root/repo && export TMPDIR=/tmp
NAME=$1; ARGS=$2; shift 2
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-global-leg --no-surface-leg --no-airplane-leg $ARGS"
for spec in "$@"; do
  v=${spec%%|*}; envs=${spec#*|}
  O=gpurun_out/$NAME/$v; mkdir -p $O
  run() { local sub=$1; shift; env $envs SRT_PIPELINE_OVERLAP=0 timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $O/$sub -o run -- $B \
            > $O/$sub.log 2>&1 || { echo "$v $sub failed"; tail -3 $O/$sub.log; exit 1; }; }
  env $envs timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-global-leg --no-surface-leg --no-airplane-leg $ARGS \
    > $O/bench.json 2> $O/bench.err || { echo "$v bench failed"; tail -3 $O/bench.err; exit 1; }
  run pmc_sq SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU
  run pmc_sq2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE
  run pmc_ta1 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
  run pmc_ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE
  run pmc_td TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
  run pmc_tcp1 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
  run pmc_tcp2 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
  run pmc_tcp3 TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_LATENCY_sum TCP_TA_TCP_STATE_READ_sum
  run pmc_tcc TCC_HIT_sum TCC_MISS_sum
  echo "$v done: $(python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['kernel_ms'])")"
done
