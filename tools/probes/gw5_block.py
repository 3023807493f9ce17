"""Probe: resident blocks per CU of the 5-wave fused instance at its build's block size (SRT_GW5_BLOCK)."""
import sys, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd")); sys.path.insert(0, str(ROOT))
from srt_amd import render as R
r = R.Renderer(R.make_setup(480, 270, show_model=True, models=[R.torus_knot_model()]))
r.render(4); r.finish()
c = r.compute
print({k: c.GetInt(k) for k in ("scene.global_waves", "scene.top_depth", "scene.top_f4", "launch.top_f4",
                                "launch.block", "launch.blocks_per_cu")})
r.close()
