"""The launch tail's single-batch window (SRT_TAIL_CLAIMS: claims per wave before the end of a launch
from which a claim takes one batch instead of kClaim) against the share of the frame a launch renders:
one GPU's whole frame, and one rank's share of an N-GPU split (row bands, srt_amd.parallel), each timed
with the library's HIP events (best of 2).  A share of an 8-GPU split has 1/8 of the batches per wave,
so a window sized for the whole frame covers a large part of its launch, where every claim is one
atomic on the launch's single counter.

Usage: python tools/probes/tail_sweep.py [scene] [spp] [band_rows] [tails, comma-separated]
"""
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))

from srt_amd import render as R  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "rubik"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
band = int(sys.argv[3]) if len(sys.argv) > 3 else 2
tails = [int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "16,8,4,2,1").split(",")]
W, H = (1920, 1080) if scene != "spheres" else (1024, 1024)
models = [R.rubik_model(ROOT / "tests" / "golden" / "objects")] if scene == "rubik" else None
setup = R.make_setup(W, H, show_model=scene == "rubik", models=models, max_depth=5 if scene == "rubik" else 4)


def kernel_ms(rank, nranks):
    r = R.Renderer(setup, rank=rank, nranks=nranks, band_rows=band)
    try:
        best = None
        for _ in range(3):
            r.render(spp, write_output=False)
            r.finish()
            ms = r.compute.last_kernel_ms()
            best = ms if best is None else min(best, ms)
        return best
    finally:
        r.close()


for t in tails:
    os.environ["SRT_TAIL_CLAIMS"] = str(t)
    one = kernel_ms(0, 1)
    parts = {n: max(kernel_ms(r, n) for r in (0, n - 1)) for n in (2, 4, 8)}
    print(f"{scene} {W}x{H} @{spp} spp tail_claims {t}: 1 GPU {one:.3f} ms | " +
          " | ".join(f"N={n} rank share {ms:.3f} ms = {one / ms / n:.3f} of linear" for n, ms in parts.items()),
          flush=True)
