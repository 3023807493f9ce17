#!/usr/bin/env python3
"""Diagnostic: how many traversal steps a shadow ray takes under the reference's child order, nearer-first
and farther-first (tools/probes/shadow_order.c), and how many fused sub-steps (memory round trips) under the
kernel's schedule and under schedules that expand the stack's top entry in the same step (tools/probes/shadow_steps.c).  Shadow rays (CheckLightOccluded) only need CheckHit(...).hit,
which does not depend on the visit order, so an any-hit walk may take either child first.

The rays: the camera ray through each pixel centre of a W x H frame of the scene (model camera), its first
hit (the oracle's closest-hit query), and from that point one shadow ray to each of the scene's lights.

  python tools/probes/shadow_order.py [torusknot|rubik] [W] [H]
"""
from __future__ import annotations

import pathlib
import subprocess
import sys
import tempfile

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))

import srt_amd as S  # noqa: E402
from srt_amd import render as R  # noqa: E402
from oracle import pyoracle as O  # noqa: E402


def main():
    scene_name = sys.argv[1] if len(sys.argv) > 1 else "torusknot"
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 480
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 270
    model = R.torus_knot_model() if scene_name == "torusknot" else R.rubik_model(ROOT / "tests/golden/objects")
    setup = R.make_setup(W, H, show_model=True, models=[model])
    sc, cam = setup.scene, setup.camera
    o = np.asarray(cam.getOrigin(), np.float32)
    right, up, front = (np.asarray(v, np.float32) for v in (cam.getRightVector(), cam.getUpVector(), cam.getForward()))
    du, dv = right / np.float32(W), up / np.float32(H)
    p00 = (o + front - right / 2 - up / 2) + 0.5 * (du + dv)
    x, y = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32))
    ps = p00 + x.reshape(-1, 1) * du + y.reshape(-1, 1) * dv
    rays = np.zeros(W * H, S.RAY_DTYPE)
    rays["o"] = o
    rays["d"] = ps - o
    rays["t"] = np.float32(np.inf)
    hits, t, _, _ = O.Oracle(sc).trace_closest(1, rays)
    m = hits != 0xFFFFFFFF
    p = rays["o"][m] + t[m, None] * rays["d"][m]
    lights = setup.lights
    lp = np.stack([lights["position"] if "position" in lights.dtype.names else lights["pos"]]).reshape(-1, 3)
    sh = []
    for L in lp:
        v = L[None, :] - p
        dist = np.linalg.norm(v, axis=1).astype(np.float32)
        sh.append(np.concatenate([p, v / dist[:, None], dist[:, None]], axis=1))
    sh = np.concatenate(sh).astype(np.float32)
    verts = sc.verts["pos"]
    tri = verts[sc.tris["v"]].reshape(-1, 9).astype(np.float32)
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([len(sc.nodes), len(tri), len(sh)], np.uint32).tobytes())
        f.write(sc.nodes.tobytes())
        f.write(tri.tobytes())
        f.write(sh.tobytes())
        path = f.name
    print(f"{scene_name} {W}x{H}: {int(m.sum())} camera-ray hits x {len(lp)} lights = {len(sh)} shadow rays")
    for tool in ("shadow_order", "shadow_steps"):  # visit orders; fused sub-steps (round trips) per schedule
        exe = pathlib.Path(tempfile.gettempdir()) / tool
        subprocess.run(["gcc", "-O2", "-o", str(exe), str(ROOT / "tools" / "probes" / f"{tool}.c"), "-lm"], check=True)
        print(subprocess.run([str(exe), path], check=True, capture_output=True, text=True).stdout, end="")
    pathlib.Path(path).unlink()


if __name__ == "__main__":
    main()
