cd /root/repo && export TMPDIR=/tmp
O=gpurun_out/wfprof; mkdir -p $O
SRT_WAVEFRONT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/torus -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-global-leg --no-surface-leg --scene torusknot --spp 64 > $O/torus.json 2> $O/torus.err || { echo torus failed; tail $O/torus.err; exit 1; }
SRT_WAVEFRONT=1 SRT_TREELETS=1 SRT_WF_SLOTS=4194304 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-global-leg --no-surface-leg --scene synthetic --width 4096 --height 4096 --spp 16 > $O/c5.json 2> $O/c5.err || { echo c5 failed; tail $O/c5.err; exit 1; }
find $O -name "*stats*"
