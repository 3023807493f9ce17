#!/bin/bash
# Round close on one box: GPU parity suite + smoke, the bench line (roofs from the committed counters of
# this code), then the other BASELINE configs (tools/configs.sh).  Outputs under gpurun_out/close/.
cd /root/repo && export TMPDIR=/tmp
O=gpurun_out/close; mkdir -p $O
bash tools/gpu_tests.sh > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -4 $O/tests.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline']['bound'])"
bash tools/configs.sh > $O/configs.log 2>&1; rc=$?; cat $O/configs.log; cp -r gpurun_out/configs $O/ 2>/dev/null; exit $rc
