"""Development probe for pool_kernel (pool.hpp): oracle parity on small Rubik frames (counting and
timed instances, per-frame dispatches), then the metric frame with and without pools, bitwise and timed.
usage: python tools/probes/pool_check.py [spp_big]   (runs with SRT_POOL toggled per context)"""
import os
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
for p in (ROOT / "simple-ray-tracer_amd", ROOT, ROOT / "tests"):
    sys.path.insert(0, str(p))
from srt_amd import render as R  # noqa: E402
from conftest import bits_equal, oracle_render  # noqa: E402


def dump_ctl(r):
    """pool_kernel's control words as the first block whose watchdog fired left them."""
    import ctypes as C

    from srt_amd import _lib

    lib = _lib.lib()
    lib.srt_debug_phase_cycles.argtypes = [C.c_void_p, C.c_void_p]
    out = np.zeros(58, np.uint64)
    lib.srt_debug_phase_cycles(r.compute.ctx, out.ctypes.data)
    names = ["headS", "headT", "headF", "tailS", "tailT", "tailF", "availS", "availT", "availF", "live", "exh", "err",
             "tid"]
    print("  watchdog state:", dict(zip(names, [int(v) for v in out[34:47]])), flush=True)


def gpu(setup, spp, pool, count=True):
    os.environ["SRT_POOL"] = "1" if pool else "0"
    r = R.Renderer(setup)
    try:
        r.render(spp, count=count)
        try:
            r.finish()
        except Exception:
            dump_ctl(r)
            raise
        t0 = time.time()
        r.render(spp, count=False)
        r.finish()
        dt = time.time() - t0
        return r.accum(), r.output(), r.compute.stats(), r.compute.last_kernel_ms(), dt
    finally:
        r.close()


def main():
    rubik = [R.rubik_model(ROOT / "tests" / "golden" / "objects")]
    for (w, h, spp) in ((64, 48, 3), (96, 72, 5), (33, 17, 2)):
        setup = R.make_setup(w, h, show_model=True, models=rubik)
        acc, out, st = oracle_render(setup, spp)
        ga, go, gst, kms, _ = gpu(setup, spp, True)
        ok = bits_equal(ga, acc).all() and (go == out).all()
        print(f"{w}x{h}@{spp}: pool parity {ok}; rays {gst['rays']} vs {st['rays']}, kernel {kms:.2f} ms", flush=True)
        if not ok:
            bad = ~bits_equal(ga, acc).all(axis=-1)
            print("  differing pixels", int(bad.sum()), "first", np.argwhere(bad)[:5].tolist(), flush=True)
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    setup = R.make_setup(1920, 1080, show_model=True, models=rubik)
    a0, o0, s0, k0, _ = gpu(setup, spp, False)
    a1, o1, s1, k1, _ = gpu(setup, spp, True)
    same = bits_equal(a0, a1).all() and (o0 == o1).all()
    print(f"1080p@{spp}: pool == sample_kernel {same}; rays {s1['rays']} vs {s0['rays']}; "
          f"kernel {k1:.2f} ms vs {k0:.2f} ms -> {s0['rays'] / k1 / 1e3:.0f} vs {s0['rays'] / k0 / 1e3:.0f} Mrays/s",
          flush=True)




def pool_stats(spp=32):
    """The -DSRT_POOL_STATS build's counters (SRT_LIB_PATH) on the metric frame."""
    import ctypes as C

    from srt_amd import _lib

    os.environ["SRT_POOL"] = "1"
    setup = R.make_setup(1920, 1080, show_model=True, models=[R.rubik_model(ROOT / "tests" / "golden" / "objects")])
    r = R.Renderer(setup)
    r.render(spp)
    r.finish()
    r.render(spp)
    r.finish()
    lib = _lib.lib()
    lib.srt_debug_phase_cycles.argtypes = [C.c_void_p, C.c_void_p]
    out = np.zeros(58, np.uint64)
    lib.srt_debug_phase_cycles(r.compute.ctx, out.ctypes.data)
    d = [float(v) for v in out[10:10 + 23]]
    names = ["T_outer", "T_inner", "T_active", "T_idle", "T_swapped", "T_hits", "T_cyc_swap", "T_cyc_trav", "T_cyc_idle",
             "S_pass", "S_popped", "S_done", "T_spare", "T_new", "S_idle", "S_cyc_busy", "S_cyc_idle", "T_wait",
             "T_c_ret", "T_c_pop", "T_c_spare", "T_c_refill", "T_c_start"]
    v = dict(zip(names, d))
    print("kernel_ms", r.compute.last_kernel_ms())
    print({k: f"{x:.4g}" for k, x in v.items()})
    tw = v["T_cyc_swap"] + v["T_cyc_trav"] + v["T_cyc_idle"]
    print(f"traversal waves: swap {v['T_cyc_swap'] / tw:.3f} trav {v['T_cyc_trav'] / tw:.3f} idle {v['T_cyc_idle'] / tw:.3f}; "
          f"active lanes per iteration {v['T_active'] / max(v['T_inner'], 1):.1f}; iterations per outer "
          f"{v['T_inner'] / max(v['T_outer'], 1):.2f}; hits {v['T_hits']:.3g} swapped {v['T_swapped']:.3g} spare "
          f"{v['T_spare']:.3g} new samples {v['T_new']:.3g}; waiting lanes per outer {v['T_wait'] / max(v['T_outer'], 1):.2f}")
    print("swap phase split:", {k: round(v[k] / max(v["T_cyc_swap"], 1), 3) for k in
                                 ("T_c_ret", "T_c_pop", "T_c_spare", "T_c_refill", "T_c_start")})
    sw = v["S_cyc_busy"] + v["S_cyc_idle"]
    print(f"shading waves: busy {v['S_cyc_busy'] / max(sw, 1):.3f}; hits per pass {v['S_popped'] / max(v['S_pass'], 1):.1f}, "
          f"paths done per pass {v['S_done'] / max(v['S_pass'], 1):.1f}")
    r.close()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "stats":
        pool_stats(int(sys.argv[1]))
    else:
        main()
