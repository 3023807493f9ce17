"""Multi-GPU load balance, measured on one GPU: each rank's share of the frame (row bands dealt
round-robin, srt_amd.parallel) is rendered on its own, one after the other, and timed with the
library's HIP events.  A node of N GPUs finishes the sample kernel when its slowest rank does, so
max over ranks of the share's kernel time predicts the N-GPU step (before the gather, which moves
W*H*16 B / N per rank).

Usage: python tools/probes/rank_shares.py [spp] [band_rows] [scene]
"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))

from srt_amd import render as R  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
band = int(sys.argv[2]) if len(sys.argv) > 2 else 8
scene = sys.argv[3] if len(sys.argv) > 3 else "rubik"
W, H = 1920, 1080
models = [R.rubik_model(ROOT / "tests" / "golden" / "objects")] if scene == "rubik" else None
setup = R.make_setup(W, H, show_model=scene == "rubik", models=models)


def share(rank, nranks):
    r = R.Renderer(setup, rank=rank, nranks=nranks, band_rows=band)
    try:
        r.render(spp, count=True, write_output=False)
        r.finish()
        rays = r.compute.stats()["rays"]
        best = None
        for _ in range(2):
            r.render(spp, write_output=False)
            r.finish()
            ms = r.compute.last_kernel_ms()
            best = ms if best is None else min(best, ms)
        return rays, best
    finally:
        r.close()


base_rays, base_ms = share(0, 1)
print(f"{scene} {W}x{H} @{spp} spp, {band}-row bands: 1 GPU {base_ms:.2f} ms, {base_rays / base_ms / 1e3:.0f} Mrays/s",
      flush=True)
for n in (2, 4, 8):
    res = [share(r, n) for r in range(n)]
    rays = sum(x[0] for x in res)
    assert rays == base_rays, (rays, base_rays)
    ms = [x[1] for x in res]
    mx, mean = max(ms), sum(ms) / n
    print(f"N={n}: per-rank kernel ms {' '.join(f'{m:.2f}' for m in ms)} | max/mean {mx / mean:.3f} | "
          f"predicted {rays / mx / 1e3:.0f} Mrays/s = {base_ms / mx / n:.3f} of linear", flush=True)
