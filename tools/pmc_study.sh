#!/bin/bash
# Counter study of one workload under several variants (runtime knobs or library builds):
#   tools/pmc_study.sh NAME "BENCH ARGS" "var1|ENV=x" "var2|ENV=y" ...
# Per variant: the timed launch's kernel time (bench.py, 3 steps) and its counters, one rocprofv3 pass per
# counter group (MI355X_MICROARCH.md: separate passes, at most 8 SQ / 4 TCC / 4 TCP counters; FETCH_SIZE
# tallies 128-B lines at 64 B on gfx950).  Reduced by tools/pmc_study.py.  Outputs: gpurun_out/$NAME/<var>/.
cd /root/repo && export TMPDIR=/tmp
# (PMC passes run their launches in series, SRT_PIPELINE_OVERLAP=0: the same kernels and work; an overlapped
# launch's counter window would also hold its wait for the CUs another launch holds, doubling its cycle counters)
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
  run pmc_fetch FETCH_SIZE
  run pmc_write WRITE_SIZE
  run pmc_tcc TCC_HIT_sum TCC_MISS_sum
  run pmc_tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
  echo "$v done: $(python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['kernel_ms'])")"
done
