# round 4 call u: pipelined launches overlapping each other (default) vs sample launches in series with
# the accumulations beside them (SRT_PIPELINE_OVERLAP=0) vs one stream (SRT_PIPELINE=1); rocprofv3's
# dispatch durations for the serial form
cd /root/repo && export TMPDIR=/tmp; O=gpurun_out/r04u; mkdir -p $O
TAG=r04u/metric REPEAT=2 BENCH_ARGS=" " bash tools/ab.sh "p3|" "p3s|SRT_PIPELINE_OVERLAP=0" "p1|SRT_PIPELINE=1" || exit 1
TAG=r04u/c2 REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene spheres --width 1024 --height 1024 --spp 64 --max-depth 4" bash tools/ab.sh "p3|" "p3s|SRT_PIPELINE_OVERLAP=0" "p1|SRT_PIPELINE=1" || exit 1
for v in "SRT_PIPELINE=1" "SRT_PIPELINE_OVERLAP=0" "SRT_PIPELINE=3"; do env $v timeout -k 10 300 python tools/pipe_probe.py 8 256 6 2>/dev/null | sed "s/^/$v /" | tee -a $O/probe.txt || exit 1; done
SRT_PIPELINE_OVERLAP=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof failed"; tail -5 $O/prof_bench.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -6 | cut -c1-200
python3 -c "import json; d=json.load(open('$O/prof_bench.json')); print('bench kernel_ms', d['roofline']['kernel_ms'], [(l['workload'], l['roofline']['kernel_ms']) for l in d['legs']])"
