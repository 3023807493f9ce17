#!/usr/bin/env python
"""Contract F against contract A on the GPU: the metric frame with GLSL's transcendentals as AMD's GPU
compilers lower them ("Tolerance"; csrc/pt_math.hpp SRT_CONTRACT_HW).

A GL driver on gfx9+ evaluates the reference's sin (raytrace_utils.glsl:28-30, behind every random number
of :44-54) as v_sin_f32(x / 2pi) and its pow (the sRGB encode, :177-184; the Fresnel terms) as
v_exp_f32(y * v_log_f32(x)).  The oracle cannot restate those instructions, so F is measured here on the
GPU: libsrt_amd.so (contract A, bit-identical to the oracle) and libsrt_amd_F.so (make CONTRACT=F, the
same kernels with the hardware instructions) each render the metric frame (Rubik 1920x1080, model
camera, 6 lights, maxDepth 5, every pixel) on frames 2.. and on the disjoint frames 2 + N.., and the
mean radiance accum/n is compared per pixel at each n in --marks:

  F           F on A's frames: shares A's primary-ray jitter (closer than a resampling by construction)
  F_disjoint  F on A' 's frames: like for like with the resampling floor A'
  A_resampled A on the next frames: the Monte-Carlo floor
  F_vs_F_resampled  F's own floor

Usage (on a GPU box): python tools/contract_f.py [--marks 16,64,256] [--out profiles/r04_contract_f.json]
Each render runs in its own process (one library per process: SRT_LIB_PATH).
TEST INFRASTRUCTURE: a measurement tool; the product library is never built with CONTRACT=F.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import subprocess
import sys
import tempfile
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "simple-ray-tracer_amd"
for p in (PKG, ROOT, ROOT / "tools"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402


def render(lib: str, first: int, marks, save: str, width: int, height: int) -> None:
    """(child process, SRT_LIB_PATH=lib) the reset frame, then frames first.. ; the mean radiance after
    each mark, saved as float32 (H, W, 3) arrays."""
    from srt_amd import render as R

    setup = R.make_setup(width, height, show_model=True,
                         models=[R.rubik_model(ROOT / "tests" / "golden" / "objects")], max_depth=5)
    r = R.Renderer(setup)
    try:
        r.clear()
        done, out = 0, {}
        for n in marks:
            r.compute.render_frames(first + done, n - done, write_output=True, count=False)
            r.finish()
            done = n
            out[f"m{n}"] = (r.accum()[..., :3] / np.float32(n)).astype(np.float32)
        from srt_amd import _lib

        out["code_hash"] = np.frombuffer(_lib.lib().srt_code_hash(), np.uint8)
    finally:
        r.close()
    np.savez(save, **out)


def measure(marks, width, height, libs=None, tmp=None) -> dict:
    """Renders A, A', F, F' in child processes and compares them (see the module doc)."""
    from contract_tolerance import compare

    libs = libs or {"A": str(PKG / "libsrt_amd.so"), "F": str(PKG / "libsrt_amd_F.so")}
    for k, v in libs.items():
        if not pathlib.Path(v).exists():
            raise SystemExit(f"{v} not built (make -C simple-ray-tracer_amd{' CONTRACT=F' if k == 'F' else ''})")
    tmp = pathlib.Path(tmp or tempfile.mkdtemp(prefix="contract_f_"))
    first2 = 2 + marks[-1]
    t0 = time.time()
    arrays, hashes = {}, {}
    for name, lib, first in (("A", libs["A"], 2), ("A_resampled", libs["A"], first2), ("F", libs["F"], 2),
                             ("F_disjoint", libs["F"], first2)):
        save = tmp / f"{name}.npz"
        env = dict(os.environ, SRT_LIB_PATH=lib, SRT_PRELOAD_TORCH="0")
        cmd = [sys.executable, __file__, "render", "--lib", lib, "--first", str(first), "--marks",
               ",".join(map(str, marks)), "--save", str(save), "--width", str(width), "--height", str(height)]
        subprocess.run(cmd, env=env, check=True, timeout=600)
        with np.load(save) as z:
            arrays[name] = {n: z[f"m{n}"].astype(np.float64) for n in marks}
            hashes[name] = bytes(z["code_hash"]).decode()
        print(f"{name} rendered ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
    base = arrays["A"]
    res = {"workload": f"rubik_{width}x{height}, model camera, 6 lights, maxDepth 5; every pixel; frames 2.. "
                       f"(A' and F_disjoint frames {first2}..)",
           "metric": "per-pixel L2 over RGB of the mean radiance accum/N between contract A (the kernel's, "
                     "bit-identical to the oracle) and X",
           "contracts": {"A": "kernel contract (libsrt_amd.so)",
                         "F": "GLSL sin/cos = v_sin/v_cos_f32(x / 2pi), pow = v_exp_f32(y * v_log_f32(x)) "
                              "(libsrt_amd_F.so, make CONTRACT=F), on A's frames",
                         "F_disjoint": "F on A_resampled's frames (like for like with A_resampled)",
                         "A_resampled": "A on the next frames: the Monte-Carlo floor"},
           "code_hash": hashes, "seconds": round(time.time() - t0, 1),
           "mean_radiance_A": {str(n): float(np.mean(np.sqrt(np.sum(base[n] ** 2, axis=-1)))) for n in marks},
           "by_spp": {}}
    for n in marks:
        r = {c: compare(base[n], arrays[c][n]) for c in ("F", "F_disjoint", "A_resampled")}
        r["F_vs_F_resampled"] = compare(arrays["F"][n], arrays["F_disjoint"][n])
        r["ratio_l2_mean_to_resampled"] = {c: r[c]["l2_mean"] / r["A_resampled"]["l2_mean"]
                                           for c in ("F", "F_disjoint", "F_vs_F_resampled")}
        res["by_spp"][str(n)] = r
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", nargs="?", default="all", choices=("all", "render"))
    ap.add_argument("--marks", default="16,64,256")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--lib")
    ap.add_argument("--first", type=int, default=2)
    ap.add_argument("--save")
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r04_contract_f.json"))
    args = ap.parse_args(argv)
    marks = [int(v) for v in args.marks.split(",")]
    if args.mode == "render":
        render(args.lib, args.first, marks, args.save, args.width, args.height)
        return None
    res = measure(marks, args.width, args.height)
    if args.out:
        pathlib.Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        pathlib.Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
    for n in marks:
        r = res["by_spp"][str(n)]
        print(n, " ".join(f"{c}: mean {r[c]['l2_mean']:.4g} p99 {r[c]['l2_p99']:.4g} max {r[c]['l2_max']:.4g} "
                          f"bias {['%.1e' % v for v in r[c]['image_mean_diff_rgb']]}"
                          for c in ("F", "F_disjoint", "A_resampled")))
    return res


if __name__ == "__main__":
    main()
