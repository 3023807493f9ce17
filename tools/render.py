"""Render a scene to an image file on the GPU: the reference's progressive loop, headless.

usage: python tools/render.py [--scene rubik|spheres|synthetic|torusknot|airplane_knot] [--width W] [--height H] [--spp N]
                              [--max-depth D] [--out frame.png]
The output is image0 after N sampled frames (src/main.cpp:642-659 accumulation schedule),
written top row first (PNG or PPM by extension).
"""
import argparse
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))

from srt_amd import render as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="rubik", choices=("rubik", "spheres", "synthetic", "torusknot", "airplane_knot"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--max-depth", type=int, default=5)
    ap.add_argument("--synthetic-tris", type=int, default=1_000_000)
    ap.add_argument("--out", default="frame.png")
    a = ap.parse_args()
    if a.scene == "rubik":
        models, show = [R.rubik_model(ROOT / "tests" / "golden" / "objects")], True
    elif a.scene == "synthetic":
        models, show = [R.synthetic_model(a.synthetic_tris)], True
    elif a.scene == "torusknot":
        models, show = [R.torus_knot_model()], True
    elif a.scene == "airplane_knot":  # the surface mesh carrying the Airplane's textured materials (bench.py leg)
        sys.path.insert(0, str(ROOT))
        import bench

        models, show = [bench.airplane_knot_model()], True
    else:
        models, show = None, False
    setup = R.make_setup(a.width, a.height, show_model=show, models=models, max_depth=a.max_depth)
    r = R.Renderer(setup)
    try:
        t0 = time.perf_counter()
        r.render(a.spp)
        r.finish()
        dt = time.perf_counter() - t0
        r.compute.save_image(a.out)
    finally:
        r.close()
    print(f"{a.out}: {a.width}x{a.height} @ {a.spp} spp in {dt:.3f} s")


if __name__ == "__main__":
    main()
