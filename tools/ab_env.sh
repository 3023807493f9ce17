#!/bin/bash
# A/B of environment knobs / library builds on the metric workload (and the global-scene leg).
# RUNS_FILE lines: "name|ENV=value ENV2=value" (e.g. SRT_LIB_PATH=..., SRT_TILE_ORDER=0)
cd /root/repo && export TMPDIR=/tmp
TAG=${TAG:-abenv}; O=gpurun_out/$TAG; mkdir -p $O
while IFS='|' read -r name envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $BENCH_ARGS \
    > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -5 $O/$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$name.json'))
g=' '.join(f\"| {l['workload']} {l['value']} Mrays/s kernel {l['roofline']['kernel_ms']}\" for l in d.get('legs', []))
print('$name', d['config']['workload'], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step, kernel', d['roofline']['kernel_ms'], g)"
done < ${RUNS_FILE:-tools/runs.txt}
