#!/bin/bash
# variant sweep: each line "NAME|ENV..." runs bench once (steps 2)
cd /root/repo && export TMPDIR=/tmp
TAG=${TAG:-sweep}; mkdir -p gpurun_out/$TAG
while IFS='|' read -r name envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/$TAG/$name.log 2> gpurun_out/$TAG/$name.err || { echo "$name FAILED"; tail -3 gpurun_out/$TAG/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/$TAG/$name.log')); print('$name', d['value'], d['ms_per_step'])"
done < ${SWEEP_FILE:-tools/runs/sweep.txt}
