"""Back-to-back renders of one rank's share (the metric workload, 2-row bands) with and without the
pipelined sample launches (SRT_PIPELINE): host wall time per render over `steps` renders enqueued
without a synchronisation between them, as bench.py's timed loop enqueues its steps.

Usage: python tools/probes/pipe_probe.py [nranks] [spp] [steps] [scene]   (run once per SRT_PIPELINE value)
"""
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))

from srt_amd import render as R  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 8
scene = sys.argv[4] if len(sys.argv) > 4 else "rubik"
if scene == "rubik":
    setup = R.make_setup(1920, 1080, show_model=True, models=[R.rubik_model(ROOT / "tests" / "golden" / "objects")])
else:
    setup = R.make_setup(1024, 1024, show_model=False, max_depth=4)
r = R.Renderer(setup, rank=0, nranks=n, band_rows=2)
try:
    for _ in range(2):
        r.render(spp, write_output=True)
    r.finish()
    t0 = time.perf_counter()
    for _ in range(steps):
        r.render(spp, write_output=True)
    r.finish()
    dt = (time.perf_counter() - t0) / steps * 1e3
    print(f"{scene} nranks {n} @{spp} spp, SRT_PIPELINE={os.environ.get('SRT_PIPELINE', 'default')}: "
          f"{dt:.3f} ms per render (last kernel {r.compute.last_kernel_ms():.3f} ms)", flush=True)
finally:
    r.close()
