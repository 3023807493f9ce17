# round 4 call s: pipelined sample launches (SRT_PIPELINE slots): the GPU suite, then per-render wall time
# of back-to-back renders (1 GPU and one rank's share of 8), then bench A/B
cd /root/repo && export TMPDIR=/tmp; O=gpurun_out/r04s; mkdir -p $O
bash tools/gpu_tests.sh > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for n in 8 1; do for p in 1 2 3; do
  SRT_PIPELINE=$p timeout -k 10 300 python tools/pipe_probe.py $n 256 6 2>/dev/null | tee -a $O/probe.txt || exit 1
done; done
for p in 1 3; do SRT_PIPELINE=$p timeout -k 10 300 python tools/pipe_probe.py 1 64 20 spheres 2>/dev/null | tee -a $O/probe.txt || exit 1; done
TAG=r04s/metric REPEAT=2 BENCH_ARGS=" " bash tools/ab.sh "p3|" "p1|SRT_PIPELINE=1" || exit 1
