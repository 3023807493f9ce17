#!/bin/bash
# Wavefront mode vs slot-pool size (kernel-trace per kernel): torus knot, 1 M soup, C5 (treelets).
cd /root/repo && export TMPDIR=/tmp
O=gpurun_out/wfslots; mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-global-leg --no-surface-leg"
for P in 4194304 16777216; do
  SRT_WAVEFRONT=1 SRT_WF_SLOTS=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/torus$P -o run -- $B --scene torusknot --spp 64 > $O/torus$P.json 2> $O/torus$P.err || { echo fail; exit 1; }
  SRT_WAVEFRONT=1 SRT_WF_SLOTS=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/soup$P -o run -- $B --scene synthetic --synthetic-tris 1000000 --spp 16 > $O/soup$P.json 2> $O/soup$P.err || { echo fail; exit 1; }
done
SRT_WAVEFRONT=1 SRT_TREELETS=1 SRT_WF_SLOTS=33554432 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c5tl -o run -- $B --scene synthetic --width 4096 --height 4096 --spp 16 > $O/c5tl.json 2> $O/c5tl.err || { echo fail; exit 1; }
for f in $O/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['roofline']['kernel_ms'])"; done
