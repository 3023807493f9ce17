#!/bin/bash
# Round profile: bench (with CPU baseline) + rocprofv3 kernel trace + HBM traffic PMC passes.
cd /root/repo && export TMPDIR=/tmp
R=${ROUND:-r01}; O=gpurun_out/$R; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write.log 2>&1
rc=$?; echo "profile exit $rc"; cat $O/bench.json; exit $rc
