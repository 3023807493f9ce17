#!/bin/bash
# A/B of library builds on the metric workload: LIBS="name=path ..." (default: base vs current),
# each runs bench.py (no CPU baseline) and, with SHARES=1, the per-rank share timing.
cd /root/repo && export TMPDIR=/tmp
TAG=${TAG:-ab}; O=gpurun_out/$TAG; mkdir -p $O
LIBS=${LIBS:-"base=simple-ray-tracer_amd/libsrt_base.so new=simple-ray-tracer_amd/libsrt_amd.so"}
for rep in 1 2; do
for kv in $LIBS; do
  name=${kv%%=*}; path=${kv#*=}
  SRT_LIB_PATH=$path timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $BENCH_ARGS \
    > $O/$name.$rep.json 2> $O/$name.$rep.err || { echo "$name FAILED"; tail -5 $O/$name.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$name.$rep.json')); print('$name', d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step, kernel', d['roofline']['kernel_ms'])"
done
done
if [ -n "$SHARES" ]; then
for kv in $LIBS; do
  name=${kv%%=*}; path=${kv#*=}
  SRT_LIB_PATH=$path timeout -k 10 400 python tools/rank_shares.py ${SHARES_SPP:-256} ${BAND:-8} > $O/$name.shares 2>&1 || { echo "$name shares FAILED"; tail -5 $O/$name.shares; exit 1; }
  echo "== $name"; cat $O/$name.shares
done
fi
