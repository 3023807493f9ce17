"""Launch-latency probe: kernel time of tiny renders (one 8x8 batch = one wave's work, 64x64, the
1080p frame) at 1 spp; the single-batch time is the latency of that wave's slowest path."""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd")); sys.path.insert(0, str(ROOT))
from srt_amd import render as R
model = R.rubik_model(ROOT / "tests" / "golden" / "objects")
for (w, h) in ((8, 8), (64, 64), (1920, 1080)):
    setup = R.make_setup(w, h, show_model=True, models=[model])
    r = R.Renderer(setup)
    for spp in (1, 4):
        ts = []
        for _ in range(5):
            r.render(spp, write_output=False); r.finish(); ts.append(r.compute.last_kernel_ms())
        r.render(spp, count=True, write_output=False); r.finish()
        st = r.compute.stats()
        print(f"{w}x{h} spp {spp}: kernel ms min {min(ts):.3f} max {max(ts):.3f}  rays {st['rays']}", flush=True)
    r.close()
