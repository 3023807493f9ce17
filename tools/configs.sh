#!/bin/bash
# BASELINE.json configs other than the metric workload, 1 GPU (Mrays/s is a rate: C5 runs fewer spp; C2, a
# 2.6-ms step, times 20 steps so the first launch, which has no predecessor to overlap, does not dominate).
cd /root/repo && export TMPDIR=/tmp
O=gpurun_out/configs; mkdir -p $O
run() { local name=$1; shift
  timeout -k 10 900 python bench.py --no-cpu-baseline --no-global-leg --no-surface-leg --no-airplane-leg "$@" > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step', 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"; }
run c2_spheres_1024_64spp_d4 --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4 --steps 20 --warmup 1 && \
run c4_rubik_4096_1024spp_d8 --scene rubik --width 4096 --height 4096 --spp 1024 --max-depth 8 --steps 1 --warmup 0 && \
run c5_synth10M_4096_16spp --scene synthetic --width 4096 --height 4096 --spp 16 --steps 1 --warmup 0
