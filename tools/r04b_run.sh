export TMPDIR=/tmp; mkdir -p gpurun_out/r04b
timeout -k 10 700 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_multirank.py tests/test_gpu_configs.py "tests/test_gpu_parity.py::test_unreachable_garbage_nodes" "tests/test_gpu_parity.py::test_surface_mesh_global_mode" "tests/test_gpu_parity.py::test_node_layouts_global_mode" tests/test_gpu_contract_f.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r04b/new.log 2>&1
echo tests_rc=$?; tail -3 gpurun_out/r04b/new.log
hipcc -O2 --offload-arch=gfx950 tools/sin_probe.hip -o /tmp/sin_probe && timeout -k 10 60 /tmp/sin_probe > gpurun_out/r04b/sin_probe.json || exit 1
TAG=r04b/ab_inl REPEAT=2 BENCH_ARGS="--no-global-leg --no-surface-leg --scene torusknot --spp 64" bash tools/ab.sh "inl1|SRT_INLINE_LEAVES=1" "inl0|SRT_INLINE_LEAVES=0" || exit 1
TAG=r04b/ab_inl1m REPEAT=1 BENCH_ARGS="--no-global-leg --no-surface-leg --scene synthetic --synthetic-tris 1000000 --spp 16" bash tools/ab.sh "inl1|SRT_INLINE_LEAVES=1" "inl0|SRT_INLINE_LEAVES=0" || exit 1
timeout -k 10 300 python tools/contract_f.py --out gpurun_out/r04b/contract_f.json > gpurun_out/r04b/contract_f.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 2 --same-device --no-cpu-baseline --steps 2 > gpurun_out/r04b/bench_g2.json 2> gpurun_out/r04b/bench_g2.err
echo rc=$?
