"""Predicted strong scaling of the metric frame from one GPU: per-render wall time of back-to-back
renders (as bench.py's timed loop enqueues its steps) of the whole frame and of the first and last
rank's share of an N-GPU split (2-row bands), at the build's defaults (launches overlap on a
multi-rank share, section 5 of DESIGN.md).  A share's time bounds its rank's step; the gather of the
sRGB8 rows (4 B/px) and the assembly on rank 0 come on top on a real node.

Usage: python tools/probes/scale_probe.py [steps] [band_rows]  (all ranks' shares at N = 8 with a third argument "all")
"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))

from srt_amd import render as R  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
band = int(sys.argv[2]) if len(sys.argv) > 2 else 2
every = len(sys.argv) > 3 and sys.argv[3] == "all"
setup = R.make_setup(1920, 1080, show_model=True, models=[R.rubik_model(ROOT / "tests" / "golden" / "objects")])


def per_render_ms(rank, n):
    r = R.Renderer(setup, rank=rank, nranks=n, band_rows=band)
    try:
        r.render(256, count=True)
        r.render(256)
        r.finish()
        t0 = time.perf_counter()
        for _ in range(steps):
            r.render(256)
        r.finish()
        return (time.perf_counter() - t0) / steps * 1e3
    finally:
        r.close()


one = per_render_ms(0, 1)
print(f"N=1: {one:.3f} ms per render ({band}-row bands)", flush=True)
for n in ((8,) if every else (2, 4, 8)):
    ranks = range(n) if every else (0, n - 1)
    ms = max(per_render_ms(r, n) for r in ranks)
    print(f"N={n}: slowest share {ms:.3f} ms per render = {one / n / ms:.3f} of linear", flush=True)
