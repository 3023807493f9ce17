"""Where an N-GPU rank share's time goes (the metric workload, 2-row bands): the share's launch against
the 1-GPU launch of the same batch count (spp / N frames of the whole image), and every rank's share
(max against mean: imbalance between ranks).  Library HIP-event kernel times, best of 3.

Usage: python tools/probes/share_probe.py [N] [band_rows]
"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))

from srt_amd import render as R  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
band = int(sys.argv[2]) if len(sys.argv) > 2 else 2
SPP = 256
setup = R.make_setup(1920, 1080, show_model=True, models=[R.rubik_model(ROOT / "tests" / "golden" / "objects")])


def kernel_ms(spp, rank, nranks):
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


full = kernel_ms(SPP, 0, 1)
part = kernel_ms(SPP // N, 0, 1)
shares = [kernel_ms(SPP, r, N) for r in range(N)]
mean = sum(shares) / N
print(f"1 GPU @{SPP} spp {full:.3f} ms; /{N} = {full / N:.3f} ms")
print(f"1 GPU @{SPP // N} spp (the share's batch count, whole-image tiles) {part:.3f} ms = {full / N / part:.3f} of linear")
print(f"rank shares @{SPP} spp, {band}-row bands: " + " ".join(f"{s:.3f}" for s in shares))
print(f"  max {max(shares):.3f} ms = {full / N / max(shares):.3f} of linear; mean {mean:.3f} ms = {full / N / mean:.3f}", flush=True)
