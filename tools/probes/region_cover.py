#!/usr/bin/env python3
"""Diagnostic: the share of a frame's node-pair loads an LDS region of K pairs serves, for the product's
depth cut, a surface-area cut and the K most-loaded pairs (tools/probes/region_cover.c).  Rays: the camera
ray through each pixel centre (model camera), one shadow ray per hit to a random light, one cosine-weighted
bounce ray per front-facing hit, and the bounce hits' shadow rays (two path segments, as the legs' paths mostly
end there).  python tools/probes/region_cover.py [knot|rubik] [W] [H]   (CPU; the oracle finds the hits)"""
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
    name = sys.argv[1] if len(sys.argv) > 1 else "knot"
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 480
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 270
    model = R.torus_knot_model() if name == "knot" else R.rubik_model(ROOT / "tests/golden/objects")
    setup = R.make_setup(W, H, show_model=True, models=[model])
    sc, cam = setup.scene, setup.camera
    orc = O.Oracle(sc)
    rng = np.random.default_rng(5)
    o = np.asarray(cam.getOrigin(), np.float32)
    right, up, front = (np.asarray(v, np.float32) for v in (cam.getRightVector(), cam.getUpVector(), cam.getForward()))
    du, dv = right / np.float32(W), up / np.float32(H)
    p00 = (o + front - right / 2 - up / 2) + 0.5 * (du + dv)
    x, y = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32))
    ps = p00 + x.reshape(-1, 1) * du + y.reshape(-1, 1) * dv
    cam_o = np.broadcast_to(o, ps.shape).astype(np.float32)
    cam_d = (ps - o).astype(np.float32)
    verts = sc.verts["pos"]
    tri = verts[sc.tris["v"]].astype(np.float32)  # (n, 3, 3), BVH order
    nrm = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True) + 1e-30
    lp = setup.lights["position"] if "position" in setup.lights.dtype.names else setup.lights["pos"]
    lp = np.asarray(lp, np.float32).reshape(-1, 3)
    out = []  # (o, d, tmax, kind)

    def closest(ro, rd):
        rays = np.zeros(len(ro), S.RAY_DTYPE)
        rays["o"], rays["d"], rays["t"] = ro, rd, np.float32(np.inf)
        out.append(np.concatenate([ro, rd, np.full((len(ro), 1), np.inf, np.float32), np.zeros((len(ro), 1), np.float32)], 1))
        h, t, _, _ = orc.trace_closest(1, rays)
        m = h != 0xFFFFFFFF
        return m, h, t

    def shadows(p):
        L = lp[rng.integers(0, len(lp), len(p))]
        v = L - p
        dist = np.linalg.norm(v, axis=1).astype(np.float32)
        out.append(np.concatenate([p, v / dist[:, None], dist[:, None], np.ones((len(p), 1), np.float32)], 1).astype(np.float32))

    ro, rd = cam_o, cam_d
    for seg in range(2):
        m, h, t = closest(ro, rd)
        p = (ro[m] + t[m, None] * rd[m]).astype(np.float32)
        shadows(p)
        n = nrm[h[m]]
        dn = rd[m] / np.linalg.norm(rd[m], axis=1, keepdims=True)
        front_facing = (n * -dn).sum(1) > 0  # brdf.glsl:242 rejects the rest
        p, n = p[front_facing], n[front_facing]
        # cosine-weighted directions about n
        u1, u2 = rng.random(len(n)), rng.random(len(n))
        r_, phi = np.sqrt(u1), 2 * np.pi * u2
        a = np.where(np.abs(n[:, :1]) > 0.9, np.array([[0, 1, 0]]), np.array([[1, 0, 0]]))
        tx = np.cross(n, a)
        tx /= np.linalg.norm(tx, axis=1, keepdims=True)
        ty = np.cross(n, tx)
        d = (tx * (r_ * np.cos(phi))[:, None] + ty * (r_ * np.sin(phi))[:, None] + n * np.sqrt(1 - u1)[:, None])
        ro, rd = p.astype(np.float32), d.astype(np.float32)
    allr = np.concatenate(out).astype(np.float32)
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([len(sc.nodes), len(tri), len(allr)], np.uint32).tobytes())
        f.write(sc.nodes.tobytes())
        f.write(tri.reshape(-1, 9).tobytes())
        f.write(allr.tobytes())
        path = f.name
    exe = pathlib.Path(tempfile.gettempdir()) / "region_cover"
    subprocess.run(["gcc", "-O2", "-o", str(exe), str(ROOT / "tools" / "probes" / "region_cover.c"), "-lm"], check=True)
    print(f"{name} {W}x{H}:", subprocess.run([str(exe), path], check=True, capture_output=True, text=True).stdout, end="")
    pathlib.Path(path).unlink()


if __name__ == "__main__":
    main()
