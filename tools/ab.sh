#!/bin/bash
# The A/B driver: bench.py under several variants, interleaved, on one box.
#
#   tools/ab.sh "base|" "pool|SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_x.so" "frac8|SRT_TRAV_FRAC16=8"
#
# Each argument is "name|ENV=value ENV2=value" (a library build via SRT_LIB_PATH, built in-tree with
# `make -C simple-ray-tracer_amd VARIANT=_x EXTRA_HIPFLAGS=-D... LIBNAME=libsrt_x.so`, or runtime knobs).
# REPEAT rounds run every variant once per round (interleaved, so box drift hits all alike); STEPS timed
# steps each; BENCH_ARGS picks the workload (default: the metric workload without legs and CPU baseline).
# Lines go to gpurun_out/$TAG/results.txt; the script stops at the first failing run.
cd /root/repo && export TMPDIR=/tmp
TAG=${TAG:-ab}; O=gpurun_out/$TAG; mkdir -p $O
ARGS=${BENCH_ARGS:---no-global-leg --no-surface-leg --no-airplane-leg}
for rep in $(seq 1 ${REPEAT:-1}); do
  for spec in "$@"; do
    name=${spec%%|*}; envs=${spec#*|}
    env $envs timeout -k 10 ${RUN_TIMEOUT:-300} python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $ARGS \
      > $O/$name.$rep.json 2> $O/$name.$rep.err || { echo "$name FAILED"; tail -5 $O/$name.$rep.err; exit 1; }
    python3 - "$O/$name.$rep.json" "$name" "$rep" <<'EOF' | tee -a $O/results.txt
import json, sys
d = json.load(open(sys.argv[1]))
legs = " ".join(f"| {l['workload']} {l['value']} kernel {l['roofline']['kernel_ms']}" for l in d.get("legs", []))
print(sys.argv[2], "rep", sys.argv[3], d["config"]["workload"], d["value"], "Mrays/s kernel",
      d["roofline"]["kernel_ms"], "ms", legs)
EOF
  done
done
