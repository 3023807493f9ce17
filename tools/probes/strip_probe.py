#!/usr/bin/env python3
"""Diagnostic: is a global-scene workload faster per ray when the image a kernel works on is a
contiguous strip rather than the whole frame?  (The proxy for an XCD-aware batch partition: each XCD's
L2 would then serve one strip's rays.)  Renders the 8 row-band shares of a 1920x1080 frame one after the
other on one GPU, as 2-row bands dealt round robin (every share spans the frame) and as 135-row bands (each
share one contiguous strip), and prints the rays per kernel time of each split.

  python tools/probes/strip_probe.py [scene: torusknot|airplane_knot|synthetic] [spp] [band rows, comma-separated: 2,135]
"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from srt_amd import render as R  # noqa: E402


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "torusknot"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    setup, wl = bench.build_setup(scene, 1920, 1080, spp, 5, 1_000_000)
    bands = [int(b) for b in sys.argv[3].split(",")] if len(sys.argv) > 3 else [2, 135]
    for band in bands:
        rays = ms = 0.0
        for rank in range(8):
            r = R.Renderer(setup, rank=rank, nranks=8, band_rows=band)
            try:
                r.render(spp, count=True, write_output=False)
                r.finish()
                rays += r.compute.stats()["rays"]
                r.compute.kernel_time()
                for _ in range(3):
                    r.render(spp, write_output=False)
                t, n = r.compute.kernel_time()
                ms += t / 3
            finally:
                r.close()
        print(f"{wl}: 8 shares of {band}-row bands: {rays / ms / 1e3:.1f} Mrays/s over the shares' kernel time "
              f"({ms:.2f} ms, {rays:.0f} rays)")


if __name__ == "__main__":
    main()
