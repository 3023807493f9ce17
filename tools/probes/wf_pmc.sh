#!/bin/bash
# Treelet scheduling on C5: L2 traffic of wf_bottom_kernel vs sample_kernel (FETCH_SIZE; TCC hits/misses).
cd /root/repo && export TMPDIR=/tmp
O=gpurun_out/wfpmc; mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-global-leg --no-surface-leg --no-airplane-leg --scene synthetic --width 4096 --height 4096 --spp 16"
export SRT_WAVEFRONT=1 SRT_TREELETS=1 SRT_WF_SLOTS=${SLOTS:-33554432}
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/tcc -o run -- $B > $O/tcc.log 2>&1
rc=$?; echo "exit $rc"; find $O -name "*counter_collection*"; exit $rc
