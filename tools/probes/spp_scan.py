"""Kernel time vs spp for the metric frame (and one rank's share): the intercept of the linear fit
is the per-launch fixed cost (fill + tail), the slope the steady-state cost per frame."""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd")); sys.path.insert(0, str(ROOT))
import numpy as np
from srt_amd import render as R
setup = R.make_setup(1920, 1080, show_model=True, models=[R.rubik_model(ROOT / "tests" / "golden" / "objects")])
for rank, n in ((0, 1), (0, 8)):
    r = R.Renderer(setup, rank=rank, nranks=n, band_rows=8)
    xs, ys = [], []
    for spp in (1, 2, 4, 8, 16, 32, 64, 128, 256):
        best = 1e30
        for _ in range(3):
            r.render(spp, write_output=False); r.finish(); best = min(best, r.compute.last_kernel_ms())
        xs.append(spp); ys.append(best)
        print(f"nranks {n} spp {spp:4d} kernel {best:8.3f} ms", flush=True)
    a, b = np.polyfit(xs[4:], ys[4:], 1)
    print(f"nranks {n}: {a:.4f} ms/frame + {b:.3f} ms fixed (fit over spp >= 16)", flush=True)
    r.render(16, count=True, write_output=False); r.finish()
    print("counting run, 16 spp:", r.compute.stats(), flush=True)
    r.close()
