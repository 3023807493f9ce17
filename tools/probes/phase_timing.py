"""Diagnostic: phase split of sample_kernel (needs the SRT_PHASE_TIMING build via SRT_LIB_PATH; the
per-sub-step lines need -DSRT_SUBSTEP_STATS too, whose atomics distort the timing)."""
import ctypes as C, sys, pathlib, os
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd")); sys.path.insert(0, str(ROOT))
import srt_amd as S
from srt_amd import render as R, _lib
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 32
scene = sys.argv[2] if len(sys.argv) > 2 else "rubik"
model = R.torus_knot_model() if scene == "torusknot" else R.rubik_model(ROOT / "tests/golden/objects")
setup = R.make_setup(1920, 1080, show_model=True, models=[model])
r = R.Renderer(setup)
r.render(spp); r.finish()
r.render(spp); r.finish()
lib = _lib.lib(); lib.srt_debug_phase_cycles.argtypes = [C.c_void_p, C.c_void_p]
import numpy as np
out = np.zeros(58, np.uint64)
lib.srt_debug_phase_cycles(r.compute.ctx, out.ctypes.data)
tot = out[:3].sum()
print("kernel_ms", r.compute.last_kernel_ms(), "refill %.1f%% trav %.1f%% shade %.1f%% iters/wave %.0f" % (
    100 * out[0] / tot, 100 * out[1] / tot, 100 * out[2] / tot, out[3] / 4096))
ti, wk, tv, lf, it, sh = (float(v) for v in out[4:10])
print("trav iters/wave %.0f  per iteration: working %.1f traversing %.1f leaf %.1f internal %.1f pop-only %.1f lanes;"
      " shading lanes/outer iter %.1f" % (ti / 4096, wk / ti, tv / ti, lf / ti, it / ti, (tv - lf - it) / ti, sh / float(out[3])))
for k in range(16):
    lanes, waves, pops = (float(v) for v in out[10 + 3 * k: 13 + 3 * k])
    if waves:
        print("  sub-step %2d: executed in %5.1f%% of iterations, %4.1f lanes when executed, %4.1f lanes pop after it"
              % (k, 100 * waves / ti, lanes / waves, pops / ti))
# ray kinds (ST_DBG_KIND, in sub-steps 14-15's slots): traversing lanes summed per traversal iteration by the kind
# of their ray, and ray starts by kind -- how much of the traversal a shadow ray and its bounce ray could share
kt = [float(v) for v in out[52:55]]
ks = [float(v) for v in out[55:58]]
if sum(kt):
    print("traversal lane-iterations: shadow %.1f%% camera %.1f%% bounce %.1f%%; ray starts: camera %.0f shadow %.0f "
          "bounce %.0f" % (100 * kt[0] / sum(kt), 100 * kt[1] / sum(kt), 100 * kt[2] / sum(kt), ks[0], ks[1], ks[2]))
