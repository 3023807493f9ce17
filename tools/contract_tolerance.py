#!/usr/bin/env python
"""Per-pixel radiance tolerance between arithmetic contracts ("Tolerance").

GLSL leaves the precision of sin/cos and the fusing of a*b+c to the implementation, and the reference's
RNG turns one ulp of a hit position into a different random number (raytrace_utils.glsl:28-54).  So
"matches the GLSL render" can only mean: the converged image is within the spread that a different,
equally valid, compiler choice produces.  This script measures that spread on the CPU oracle's contract
variants (oracle/srt_oracle.c ORACLE_CONTRACT):

  A  the kernel's contract (the HIP path equals it bit for bit: tests/test_gpu_*.py)
  B  no FMA anywhere in expressions          C  every a*b+c fused (gcc -ffp-contract=fast -mfma)
  D  sin/cos in double, rounded to float     E  B + D (the round-1 contract)
  A' the kernel's contract on the next `spp` frames: an independent resampling of every pixel, the
     Monte-Carlo floor any two renders with different random numbers sit at

on the metric frame (Rubik 1920x1080, model camera, 6 lights, maxDepth 5), every `--row-step`-th row,
and reports per-pixel L2 of the mean radiance accum/N between A and each other render (mean, p50, p99,
max), the image-mean difference per channel with its standard error, at several sample counts.

Two comparisons per variant X:
  X           X on A's own frames (2..): the primary rays' jitter and, until the paths part, every random
              number are shared with A, so X sits closer to A than a resampling does by construction;
  X_disjoint  X on the next frames (2 + N..), A' 's frames: like for like with A', so any excess of
              X_disjoint over A' (L2) or any image-mean offset beyond its standard error is the
              contract's own effect (--no-disjoint skips these).

TEST INFRASTRUCTURE: it runs the oracle only (no GPU).  Output: JSON (default profiles/r04_contract_tolerance.json).
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in (ROOT / "simple-ray-tracer_amd", ROOT, ROOT / "tests"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402


def render_rows(setup, contract, rows, frame_first, spp_marks, threads):
    """Mean radiance (len(rows), W, 3) after each count in spp_marks, frames frame_first.. in order."""
    from oracle import pyoracle as O

    s = setup
    orc = O.Oracle(s.scene, s.lights, s.noise, s.noise_u, contract=contract)
    cam = s.camera
    f = O.Oracle.frame(s.width, s.height, show_model=s.show_model, bvh_count=s.bvh_count, light_count=len(s.lights),
                       max_depth=s.max_depth, origin=cam.position, direction=cam.front, up=cam.up, right=cam.right)
    acc = np.zeros((s.height, s.width, 4), np.float32)
    out = np.zeros((s.height, s.width, 4), np.uint8)
    means, done, rays = {}, 0, 0
    for n in spp_marks:
        st = orc.render_rows(f, frame_first + done, n - done, acc, out, rows, threads)
        rays += st["rays"]
        done = n
        means[n] = (acc[rows, :, :3] / np.float32(n)).astype(np.float64)
    return means, rays


def compare(a: np.ndarray, b: np.ndarray) -> dict:
    d = a - b
    l2 = np.sqrt(np.sum(d * d, axis=-1)).ravel()
    npx = l2.size
    dm = d.reshape(-1, 3)
    return {
        "l2_mean": float(l2.mean()), "l2_p50": float(np.percentile(l2, 50)),
        "l2_p99": float(np.percentile(l2, 99)), "l2_max": float(l2.max()),
        "frac_pixels_identical": float(np.mean(l2 == 0.0)),
        "image_mean_diff_rgb": [float(v) for v in dm.mean(axis=0)],
        "image_mean_diff_stderr_rgb": [float(v) for v in dm.std(axis=0) / np.sqrt(npx)],
    }


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--row-step", type=int, default=8)
    ap.add_argument("--spp", default="16,64,256")
    ap.add_argument("--contracts", default="B,C,D,E")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--no-disjoint", action="store_true")
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r04_contract_tolerance.json"))
    args = ap.parse_args(argv)
    from srt_amd import render as R

    marks = [int(v) for v in args.spp.split(",")]
    setup = R.make_setup(args.width, args.height, show_model=True,
                         models=[R.rubik_model(ROOT / "tests" / "golden" / "objects")], max_depth=5)
    rows = np.arange(0, args.height, args.row_step, dtype=np.int32)
    threads = args.threads or min(16, os.cpu_count() or 1)
    t0 = time.time()
    base, rays_a = render_rows(setup, "A", rows, 2, marks, threads)
    renders = {}
    for c in args.contracts.split(","):
        renders[c], _ = render_rows(setup, c, rows, 2, marks, threads)
        if not args.no_disjoint:
            renders[c + "_disjoint"], _ = render_rows(setup, c, rows, 2 + marks[-1], marks, threads)
        print(f"contract {c} done ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
    # A': the same contract on the next frames (an independent resampling of every pixel)
    renders["A_resampled"], _ = render_rows(setup, "A", rows, 2 + marks[-1], marks, threads)
    res = {"workload": f"rubik_{args.width}x{args.height}, model camera, 6 lights, maxDepth 5; rows 0::{args.row_step} "
                       f"({len(rows)} rows x {args.width} px); frames 2.. (A' frames {2 + marks[-1]}..)",
           "metric": "per-pixel L2 over RGB of the mean radiance accum/N between contract A (the kernel's) and X",
           "contracts": {"A": "kernel contract (dot/cross fused, fp32 FMA sin/cos)",
                         "B": "no FMA in any expression", "C": "every a*b+c fused (gcc -ffp-contract=fast -mfma)",
                         "D": "sin/cos in double rounded to float", "E": "B + D (the round-1 contract)",
                         "A_resampled": "contract A, next frames: Monte-Carlo resampling floor",
                         "X_disjoint": "contract X on A_resampled's frames: like-for-like with A_resampled"},
           "rays_A": int(rays_a), "seconds": round(time.time() - t0, 1),
           "mean_radiance_A": {str(n): float(np.mean(np.sqrt(np.sum(base[n] ** 2, axis=-1)))) for n in marks},
           "by_spp": {}}
    for n in marks:
        res["by_spp"][str(n)] = {c: compare(base[n], renders[c][n]) for c in renders}
        res["by_spp"][str(n)]["ratio_l2_mean_to_resampled"] = {
            c: res["by_spp"][str(n)][c]["l2_mean"] / res["by_spp"][str(n)]["A_resampled"]["l2_mean"] for c in renders}
    pathlib.Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
    for n in marks:
        r = res["by_spp"][str(n)]
        print(n, " ".join(f"{c}: mean {r[c]['l2_mean']:.4g} p99 {r[c]['l2_p99']:.4g} max {r[c]['l2_max']:.4g}"
                          for c in renders))
    return res


if __name__ == "__main__":
    main()
