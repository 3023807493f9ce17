# round 4 call t: pipelined launches with per-launch spans: GPU suite, bench A/B (SRT_PIPELINE 3 vs 1),
# the rank-share probe, and rocprofv3's kernel durations against bench's kernel_ms
cd /root/repo && export TMPDIR=/tmp; O=gpurun_out/r04t; mkdir -p $O
bash tools/gpu_tests.sh > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
TAG=r04t/metric REPEAT=2 BENCH_ARGS=" " bash tools/ab.sh "p3|" "p1|SRT_PIPELINE=1" || exit 1
TAG=r04t/c2 REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "p3|" "p1|SRT_PIPELINE=1" || exit 1
for p in 1 3; do SRT_PIPELINE=$p timeout -k 10 300 python tools/pipe_probe.py 8 256 6 2>/dev/null | tee -a $O/probe.txt || exit 1; done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof failed"; tail -5 $O/prof_bench.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-200
python3 -c "import json; d=json.load(open('$O/prof_bench.json')); print('bench kernel_ms', d['roofline']['kernel_ms'], [(l['workload'], l['roofline']['kernel_ms']) for l in d['legs']])"
