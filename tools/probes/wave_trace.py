"""Per-wave timeline of one sample_kernel launch (diagnostic build with -DSRT_WAVE_TRACE, loaded via
SRT_LIB_PATH): start, scene copied to LDS, batches exhausted, end -- s_memrealtime at 100 MHz."""
import ctypes as C, pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd")); sys.path.insert(0, str(ROOT))
import numpy as np
from srt_amd import render as R, _lib
lib = _lib.lib()
lib.srt_debug_wave_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
setup = R.make_setup(1920, 1080, show_model=True, models=[R.rubik_model(ROOT / "tests" / "golden" / "objects")])
CASES = {"default": [(1, 1), (1, 16), (1, 256), (8, 256)], "short": [(1, 256), (8, 256)],
         "fixed": [(1, 256), (1, 32), (8, 256)]}
for n, spp in CASES[sys.argv[1] if len(sys.argv) > 1 else "default"]:
    r = R.Renderer(setup, rank=0, nranks=n, band_rows=2)
    r.render(spp, write_output=False); r.finish()
    r.render(spp, write_output=False); r.finish()
    ms = r.compute.last_kernel_ms()
    buf = np.zeros((16384, 4), np.uint64)
    k = lib.srt_debug_wave_trace(r.compute.ctx, buf.ctypes.data, 16384)
    t = (buf[:k].astype(np.float64) - float(buf[:k, 0].min())) / 100.0  # us
    q = lambda v: " ".join(f"{x:8.1f}" for x in np.percentile(v, [0, 10, 50, 90, 99, 100]))
    print(f"nranks {n} spp {spp}: kernel {ms:.3f} ms, {k} waves; percentiles 0/10/50/90/99/100 in us from first start")
    print("  start     ", q(t[:, 0]))
    print("  lds ready ", q(t[:, 1]))
    ex = t[:, 2][buf[:k, 2] > 0]
    print("  exhausted ", q(ex) if len(ex) else "-")
    print("  end       ", q(t[:, 3]))
    print("  end - exhausted", q((t[:, 3] - t[:, 2])[buf[:k, 2] > 0]), flush=True)
    end = t[:, 3].max()
    # waves still running at each tenth of the launch, and the launch's wave-time lost to idle SIMD slots
    print("  running at 10..100% of the launch:",
          " ".join(f"{(t[:, 3] >= f * end).mean():.3f}" for f in np.arange(0.1, 1.01, 0.1)))
    print(f"  idle wave-time after each wave's end: {((end - t[:, 3]).sum() / (k * end)):.4f} of the launch;"
          f" before its start: {(t[:, 0].sum() / (k * end)):.4f}; LDS copy: {((t[:, 1] - t[:, 0]).sum() / (k * end)):.4f}",
          flush=True)
    r.close()
