#!/bin/bash
# C2 (sphere scene 1024x1024 @64 spp, maxDepth 4) at 3..6 sphere_kernel blocks per CU (SRT_SPHERE_BLOCKS):
# the timed launch's kernel time (bench.py, 3 steps) and its counters, one rocprofv3 pass per counter group
# (MI355X_MICROARCH.md: separate passes; FETCH_SIZE tallies 128-B lines at 64 B on gfx950).  Reduced by
# tools/c2_study.py into profiles/r04_c2_study.json.  Outputs under gpurun_out/c2s/b<N>/.
cd /root/repo && export TMPDIR=/tmp
# (PMC passes run their launches in series, SRT_PIPELINE_OVERLAP=0: the same kernels and work; an overlapped
# launch's counter window would also hold its wait for the CUs another launch holds, doubling its cycle counters)
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-global-leg --no-surface-leg --no-airplane-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4"
for n in ${BLOCKS:-3 4 5 6}; do
  O=gpurun_out/c2s/b$n; mkdir -p $O
  export SRT_SPHERE_BLOCKS=$n
  timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-global-leg --no-surface-leg --no-airplane-leg --scene spheres \
    --width 1024 --height 1024 --spp 64 --max-depth 4 > $O/bench.json 2> $O/bench.err || exit 1
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
    SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $O/pmc_sq -o run -- $B > $O/pmc_sq.log 2>&1 || exit 1
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
    --output-format csv -d $O/pmc_sq2 -o run -- $B > $O/pmc_sq2.log 2>&1 || exit 1
  # cycle-weighted VALU: the quad-cycles waves spend executing VALU instructions (a slow instruction -- the f64
  # multiplies of pow(x, 5), v_rcp/v_sqrt/v_sin, the v_div_* sequences -- weighs its cycles, not 1)
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 \
    SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d $O/pmc_cyc -o run -- $B > $O/pmc_cyc.log 2>&1 || exit 1
  [ -n "$CYC_ONLY" ] && { echo "b$n cyc done"; continue; }
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || exit 1
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || exit 1
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_tcc -o run -- $B > $O/pmc_tcc.log 2>&1 || exit 1
  SRT_PIPELINE_OVERLAP=0 timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum --output-format csv \
    -d $O/pmc_tcp -o run -- $B > $O/pmc_tcp.log 2>&1 || exit 1
  echo "b$n done: $(python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['kernel_ms'])")"
done
