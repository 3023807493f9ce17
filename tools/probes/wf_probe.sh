#!/bin/bash
# Wavefront mode: its GPU parity tests, then an A/B of the global-scene workloads with it on and off.
cd /root/repo && export TMPDIR=/tmp
O=gpurun_out/wf; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -x -v --timeout 200 --timeout-method thread \
  > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
run() {  # name, env, bench args
  env $2 timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-global-leg --no-surface-leg --no-airplane-leg $3 \
    > $O/$1.json 2> $O/$1.err || { echo "$1 FAILED"; tail -5 $O/$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$1.json')); print('$1', d['config']['workload'], d['value'], 'Mrays/s kernel', d['roofline']['kernel_ms'], 'ms')" | tee -a $O/results.txt
}
for rep in ${REPS:-1 2}; do
  run torus_mk$rep "SRT_WAVEFRONT=0" "--scene torusknot --spp 64"
  run torus_wf$rep "SRT_WAVEFRONT=1" "--scene torusknot --spp 64"
  run soup_mk$rep "SRT_WAVEFRONT=0" "--scene synthetic --synthetic-tris 1000000 --spp 16"
  run soup_wf$rep "SRT_WAVEFRONT=1" "--scene synthetic --synthetic-tris 1000000 --spp 16"
done
C5="--scene synthetic --width 4096 --height 4096 --spp 16 --steps 1"
run c5_mk "SRT_WAVEFRONT=0" "$C5"
run c5_wf "SRT_WAVEFRONT=1 SRT_TREELETS=0" "$C5"
run c5_tl4M "SRT_WAVEFRONT=1 SRT_TREELETS=1 SRT_WF_SLOTS=4194304" "$C5"
run c5_tl16M "SRT_WAVEFRONT=1 SRT_TREELETS=1 SRT_WF_SLOTS=16777216" "$C5"
run c5_tl16M_d12 "SRT_WAVEFRONT=1 SRT_TREELETS=1 SRT_WF_SLOTS=16777216 SRT_TREELET_DEPTH=12" "$C5"
