#!/usr/bin/env python3
"""Diagnostic: what sampling the Airplane's textures per hit costs on the surface mesh (bench.py's
airplane_materials leg).  The same OBJ (outward faces, six materials) is loaded twice: with its uvs (every
hit samples its texture: the TEX instance) and without (the reference's loader: uv = (0,0), one constant
albedo per material).  Prints the sample-kernel time per render (srt_kernel_time, 3 renders back to back)
and the counted rays of each.

  python tools/probes/airplane_probe.py [spp]
"""
import pathlib
import shutil
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))

import srt_amd as S  # noqa: E402
from srt_amd import render as R  # noqa: E402
import bench  # noqa: E402


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    with tempfile.TemporaryDirectory() as d:
        d = pathlib.Path(d)
        for f in (ROOT / "tests" / "golden" / "objects" / "11803_Airplane_v1_l1").iterdir():
            shutil.copy(f, d / f.name)
        obj = R.write_textured_torus_knot_obj(d / "k.obj", "11803_Airplane_v1_l1.mtl", bench.AIRPLANE_MATERIALS)
        models = {"textures sampled per hit": S.load_obj(obj, texcoords=True), "constant albedo (uv = 0)": S.load_obj(obj)}
    for name, m in models.items():
        setup = R.make_setup(1920, 1080, show_model=True, models=[m])
        r = R.Renderer(setup)
        try:
            r.render(spp, count=True)
            r.finish()
            rays = r.compute.stats()["rays"]
            r.compute.kernel_time()
            for _ in range(3):
                r.render(spp)
            ms, n = r.compute.kernel_time()
        finally:
            r.close()
        print(f"{name}: {ms / 3:.3f} ms per render ({n} launches), {rays} rays, {rays * 3 / ms / 1e3:.1f} Mrays/s")


if __name__ == "__main__":
    main()
