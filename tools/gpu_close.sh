#!/bin/bash
# Round closing run on one box: GPU suite + smoke, tools/profile_round.sh (bench line, kernel trace, PMC
# passes), counters.json from those passes, then the bench line that reports them.
cd /root/repo && export TMPDIR=/tmp
R=${ROUND:-r02}; O=gpurun_out/$R; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
ROUND=$R bash tools/profile_round.sh || exit 1
python tools/pmc_roofline.py $O --tag $R && cp profiles/counters.json $O/counters.json && \
timeout -k 10 600 python bench.py > $O/bench_final.json 2> $O/bench_final.err
rc=$?; echo "close exit $rc"; cat $O/bench_final.json; exit $rc
