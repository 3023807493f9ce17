"""The global-scene fused instance's LDS top region for a scene: depth, float4 laid out, float4 the last
launch copied, resident blocks per CU.  python tools/probes/top_region.py [knot|airplane|synthetic]
(SRT_LIB_PATH / SRT_TOP_BFS / SRT_TOP_DEPTH select the variant; GPU)."""
import sys

sys.path[:0] = [".", "simple-ray-tracer_amd", "tests"]
import bench  # noqa: E402
from srt_amd import render as R  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "torusknot"
setup, name = bench.build_setup(scene, 320, 180, 2, 5, 1000000)
r = R.Renderer(setup)
try:
    r.render(2)
    r.finish()
    c = r.compute
    print(name, {k: c.GetInt(k) for k in ("scene.fused", "scene.global_waves", "scene.top_depth", "scene.top_f4",
                                          "launch.top_f4", "launch.blocks_per_cu", "launch.block")})
finally:
    r.close()
