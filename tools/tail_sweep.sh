#!/bin/bash
# Tail-window sweep: SRT_TAIL_CLAIMS (claims per wave before the end from which a claim is one batch).
# Per value: the wave timeline (traced build) at N=1 and one rank of N=8, and the 1-GPU bench.
cd /root/repo && export TMPDIR=/tmp
O=gpurun_out/tail; mkdir -p $O
for F in ${TAILS:-2 8 16 32}; do
  SRT_TAIL_CLAIMS=$F SRT_LIB_PATH=simple-ray-tracer_amd/libsrt_tr.so timeout -k 10 300 python tools/wave_trace.py short \
    > $O/wt_$F.log 2>&1 || { echo "trace $F failed"; tail -5 $O/wt_$F.log; exit 1; }
  echo "== SRT_TAIL_CLAIMS=$F"; grep -A5 "spp 256" $O/wt_$F.log | grep "kernel\|exhausted  \|end  "
  SRT_TAIL_CLAIMS=$F timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$F.json 2> $O/bench_$F.err \
    || { echo "bench $F failed"; tail -5 $O/bench_$F.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$F.json')); print('bench', d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step, kernel', d['roofline']['kernel_ms'])"
done
