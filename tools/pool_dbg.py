import os, sys, pathlib, ctypes as C, numpy as np
ROOT = pathlib.Path('/root/repo')
for p in (ROOT / "simple-ray-tracer_amd", ROOT, ROOT / "tests"): sys.path.insert(0, str(p))
os.environ["SRT_POOL"] = "1"; os.environ["SRT_POOL_DEADLINE_MS"] = "3000"
from srt_amd import render as R, _lib
setup = R.make_setup(64, 48, show_model=True, models=[R.rubik_model(ROOT / "tests/golden/objects")])
r = R.Renderer(setup)
r.render(3, count=(len(sys.argv) > 1))
rc = _lib.lib().srt_finish(r.compute.ctx)
print("finish rc", rc)
lib = _lib.lib(); lib.srt_debug_phase_cycles.argtypes = [C.c_void_p, C.c_void_p]
out = np.zeros(58, np.uint64); lib.srt_debug_phase_cycles(r.compute.ctx, out.ctypes.data)
ctl = out[10 + 24: 10 + 24 + 13]
names = ["headS","headT","headF","tailS","tailT","tailF","availS","availT","availF","live","exh","err","tid"]
print(dict(zip(names, [int(v) for v in ctl])))
