"""Quick GPU-vs-oracle parity probe (development helper)."""
import sys, time, pathlib, numpy as np
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'simple-ray-tracer_amd')); sys.path.insert(0, str(ROOT))
import srt_amd as S
from srt_amd import render as R
from oracle import pyoracle as O

def oracle_render(setup, spp):
    s = setup
    orc = O.Oracle(s.scene, s.lights, s.noise, s.noise_u)
    cam = s.camera
    f = O.Oracle.frame(s.width, s.height, show_model=s.show_model, bvh_count=s.bvh_count, light_count=len(s.lights),
                       max_depth=s.max_depth, origin=cam.position, direction=cam.front, up=cam.up, right=cam.right)
    acc = np.zeros((s.height, s.width, 4), np.float32); out = np.zeros((s.height, s.width, 4), np.uint8)
    f.reset = 1; f.accum_frames = 1; orc.dispatch(f, acc, out); f.reset = 0
    st = orc.render(f, 2, spp, acc, out)
    return acc, out, st

def run(kind, W, H, spp, gpu=True):
    models = [R.rubik_model(str(ROOT / 'tests/golden/objects'))] if kind == 'rubik' else None
    setup = R.make_setup(W, H, show_model=(kind == 'rubik'), models=models)
    t0 = time.time(); acc, out, st = oracle_render(setup, spp); t1 = time.time()
    print(kind, W, H, spp, 'oracle', round(t1 - t0, 2), 's', st)
    if not gpu: return
    r = R.Renderer(setup)
    r.render(spp, count=True); r.finish()
    ga, go = r.accum(), r.output()
    print(' gpu stats', r.compute.stats())
    eq = (ga.view(np.uint32) == acc.view(np.uint32)).all(axis=-1)
    print(' accum bit-exact pixels: %d / %d' % (eq.sum(), eq.size), ' out equal:', (go == out).all(),
          ' max abs diff', float(np.nanmax(np.abs(ga - acc))))
    # per-frame Dispatch path
    r2 = R.Renderer(setup); r2.clear()
    for _ in range(spp): r2.frame()
    r2.finish(); eq2 = (r2.accum().view(np.uint32) == acc.view(np.uint32)).all()
    print(' dispatch path bit-exact:', eq2, (r2.output() == out).all())
    r.close(); r2.close()

if __name__ == '__main__':
    gpu = '--cpu' not in sys.argv
    run('spheres', 64, 64, 2, gpu)
    run('rubik', 64, 64, 2, gpu)
    run('rubik', 120, 72, 6, gpu)
    run('spheres', 72, 120, 4, gpu)
