"""GPU parity: the HIP path tracer (through the C ABI) vs the CPU oracle, bit for bit.

Bar: accumulation image bit-identical (NaN == NaN), RGBA8 image identical, CheckHit query
counts identical, on seeded inputs small enough for the oracle; at BASELINE's full frame
size, oracle rows sampled across the frame plus size-independent properties
(determinism, chunking / LDS / tiling invariance).
"""
import os
import pathlib
import subprocess

import numpy as np
import pytest

import srt_amd as S
from srt_amd import render as R
from conftest import OBJECTS, PKG, ROOT, bits_equal, oracle_render
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rubik():
    return S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")


def gpu_render(setup, spp, *, per_frame=False, timed=True, **kw):
    """The frame through the counting instance of sample_kernel (fused launch, with CheckHit counts) or
    per-frame dispatches; with `timed`, the fused launch is rendered again through the timed instance the
    benchmark measures (in global-scene mode another schedule: fused sub-steps, more waves per SIMD), which
    must give the same frame bit for bit."""
    r = R.Renderer(setup, **kw)
    try:
        if per_frame:
            r.clear()
            for _ in range(spp):
                r.frame()
        else:
            r.render(spp, count=True)
        r.finish()
        acc, out, st = r.accum(), r.output(), r.compute.stats()
        if timed and not per_frame:
            r.render(spp)
            r.finish()
            eq = bits_equal(r.accum(), acc)
            assert eq.all(), f"timed instance: {(~eq).sum()} accumulation values differ from the counting instance"
            assert (r.output() == out).all()
        return acc, out, st
    finally:
        r.close()


def assert_parity(setup, spp, **kw):
    acc, out, st = oracle_render(setup, spp)
    gacc, gout, gst = gpu_render(setup, spp, **kw)
    eq = bits_equal(gacc, acc)
    assert eq.all(), f"{(~eq).sum()} accumulation values differ"
    assert (gout == out).all()
    if not kw.get("per_frame"):
        assert gst["rays"] == st["rays"] and gst["samples"] == st["samples"]
        assert gst["shadow_rays"] == st["shadow_rays"]   # srt_ray_kinds against the oracle's count
        assert gst["stack_overflow"] == 0
    return gacc, gout


@pytest.mark.parametrize("w,h,spp,depth", [(64, 64, 2, 5), (72, 40, 3, 5), (40, 72, 2, 8), (33, 17, 2, 0)])
def test_spheres_parity(w, h, spp, depth):
    assert_parity(R.make_setup(w, h, show_model=False, max_depth=depth), spp)


@pytest.mark.parametrize("w,h,spp,depth", [(64, 64, 2, 5), (96, 54, 4, 5), (40, 72, 2, 3), (31, 23, 3, 8)])
def test_rubik_parity(rubik, w, h, spp, depth):
    assert_parity(R.make_setup(w, h, show_model=True, models=[rubik], max_depth=depth), spp)


def test_per_frame_dispatch_matches_fused(rubik):
    setup = R.make_setup(48, 40, show_model=True, models=[rubik])
    acc_f, out_f = assert_parity(setup, 3)
    acc_d, out_d, _ = gpu_render(setup, 3, per_frame=True)
    assert bits_equal(acc_d, acc_f).all() and (out_d == out_f).all()


def test_partial_dispatch_extent(rubik):
    """glDispatchCompute(gx, gy) covers only gx*8 x gy*8 invocations; other pixels keep their values."""
    setup = R.make_setup(48, 40, show_model=True, models=[rubik])
    acc, out, _ = oracle_render(setup, 1)
    r = R.Renderer(setup)
    try:
        r.clear()
        r.compute.write_accum(np.full((40, 48, 4), 7.0, np.float32))
        c = r.compute
        c.SetBool("resetAccumBuffer", True)
        c.SetInt("accumFrames", 1)
        c.Dispatch(3, 2)  # 24 x 16 pixels reset
        c.SetBool("resetAccumBuffer", False)
        c.SetInt("accumFrames", 2)
        c.Dispatch(3, 2)
        c.Finish()
        g = c.read_accum()
    finally:
        r.close()
    assert bits_equal(g[:16, :24], acc[:16, :24]).all()
    assert (g[16:, :] == 7.0).all() and (g[:, 24:] == 7.0).all()


def test_lights_edge_cases(rubik):
    # lightCount larger than the SSBO (indices past it read zeros) and a single light
    setup = R.make_setup(40, 32, show_model=True, models=[rubik])
    assert_parity(setup, 2)
    one = R.make_setup(40, 32, show_model=True, models=[rubik], lights=S.MODEL_LIGHTS[:1])
    assert_parity(one, 2)
    none = R.make_setup(32, 24, show_model=False, lights=())
    assert_parity(none, 2)


@pytest.mark.parametrize("scene", ["rubik", "knot", "spheres"])
def test_many_lights_read_from_hbm(rubik, scene):
    """300 point lights (9.6 KB of records, past the 8-KB LDS cap: shading reads them from HBM, kp.lights_lds
    = 0) through SampleLights' RIS loop of 300 iterations (raytrace_compute.glsl:179-206), whose
    randLightIndex = round(u * lightCount) can reach lightCount, one past the records (the zero light, as an
    SSBO read past its end returns): the LDS kernel (Rubik), the fused 5-wave global instance (the knot) and
    the sphere kernel match the oracle."""
    rng = np.random.default_rng(300)
    lights = [S.PointLight(tuple(rng.uniform((-12, 0, -12), (12, 22, 20)).astype(np.float32)),
                           tuple(rng.uniform(0.1, 1.0, 3).astype(np.float32)), float(np.float32(rng.uniform(1, 40))))
              for _ in range(300)]
    models = {"rubik": [rubik], "knot": [R.torus_knot_model()], "spheres": None}[scene]
    setup = R.make_setup(32, 24, show_model=scene != "spheres", models=models, lights=lights)
    assert len(setup.lights) == 300
    assert_parity(setup, 2)


def test_ghost_bvh_count(rubik):
    """src/main.cpp:683 sets bvh_count = 2 with one model: bvhs[1] is an out-of-bounds (zero) record."""
    setup = R.make_setup(40, 32, show_model=True, models=[rubik], bvh_count=2)
    acc2, out2 = assert_parity(setup, 2)
    setup1 = R.make_setup(40, 32, show_model=True, models=[rubik], bvh_count=1)
    acc1, _, _ = gpu_render(setup1, 2)
    assert bits_equal(acc1, acc2).all()  # the zero record never hits


def test_two_models_with_transform(rubik):
    second = S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")
    setup = R.make_setup(48, 40, show_model=True, models=[rubik, second])
    # move the second cube: world -> model frame translates by (-12, 2, 5)
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (12.0, -2.0, -5.0)  # glm column 3 = translation
    setup.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(setup, 2)


def _coincident_obj(tmp_path):
    """A floor (y = 0) and a back wall (z = -6), each a 4x4 grid of quads written three times: 'red' and 'green'
    are the same triangles (identical centroids, so the midpoint split keeps each twin pair in one leaf), 'blue'
    is the grid shifted by half a cell inside the same plane (coplanar overlaps in other leaves).  Every hit on
    them is a distance tie that only the visit order settles: `t < intersection_distance` is strict
    (ray_intersects.glsl:89), so the first triangle the reference's traversal reaches keeps the hit."""
    (tmp_path / "m.mtl").write_text("newmtl red\nKd 0.9 0.1 0.1\nKs 0.2 0.2 0.2\nNs 20\n"
                                    "newmtl green\nKd 0.1 0.9 0.1\nKs 0.5 0.5 0.5\nNs 80\n"
                                    "newmtl blue\nKd 0.1 0.1 0.9\nKs 0.05 0.05 0.05\nNs 5\n")
    lines, nv = ["mtllib m.mtl"], 0

    def grid(corner, du, dv, n=4):
        nonlocal nv
        base = nv
        for j in range(n + 1):
            for i in range(n + 1):
                p = np.asarray(corner, np.float64) + i * np.asarray(du) + j * np.asarray(dv)
                lines.append("v %.6g %.6g %.6g" % tuple(p))
                nv += 1
        return [(base + j * (n + 1) + i + 1, base + j * (n + 1) + i + 2, base + (j + 1) * (n + 1) + i + 2,
                 base + (j + 1) * (n + 1) + i + 1) for j in range(n) for i in range(n)]

    floor = grid((-8, 0, -8), (4, 0, 0), (0, 0, 4))
    wall = grid((-8, 0, -6), (4, 0, 0), (0, 3.5, 0))
    floor_b = grid((-6, 0, -6), (4, 0, 0), (0, 0, 4))
    wall_b = grid((-6, 1.75, -6), (4, 0, 0), (0, 3.5, 0))
    for mtl, quads in (("red", floor + wall), ("green", floor + wall), ("blue", floor_b + wall_b)):
        lines.append("usemtl " + mtl)
        lines += ["f %d %d %d %d" % q for q in quads]
    (tmp_path / "m.obj").write_text("\n".join(lines) + "\n")
    return tmp_path / "m.obj"


@pytest.mark.parametrize("mode", ["lds", "global"])
def test_coincident_triangles_keep_the_first_visited(tmp_path, monkeypatch, mode):
    """Distance ties decided by visit order, in the renderer (both scene modes, counting and timed instances)
    and in srt_trace_closest: identical twin triangles in one leaf, coplanar overlaps across leaves, and shadow
    rays leaving the plane they start on.  The oracle's order is the reference's (ray_intersects.glsl:99-133),
    so any reordering of a leaf's triangles or of sibling visits shows up as another material's colour."""
    if mode == "global":
        monkeypatch.setenv("SRT_FORCE_GLOBAL_SCENE", "1")
    model = S.load_obj(_coincident_obj(tmp_path))
    setup = R.make_setup(64, 48, show_model=True, models=[model])
    sc = setup.scene
    assert len(sc.tris) == 3 * 2 * 32
    assert_parity(setup, 3)

    rng = np.random.default_rng(17)
    n = 4096
    rays = np.zeros(n, S.RAY_DTYPE)
    rays["o"] = rng.uniform([-7, 0.5, -5], [7, 12, 6], size=(n, 3)).astype(np.float32)
    tgt = np.where((np.arange(n) % 2 == 0)[:, None],
                   np.stack([rng.uniform(-7, 7, n), np.zeros(n), rng.uniform(-7, 7, n)], 1),     # the floor
                   np.stack([rng.uniform(-7, 7, n), rng.uniform(0, 13, n), np.full(n, -6.0)], 1))  # the wall
    rays["d"] = (tgt - rays["o"]).astype(np.float32)
    rays["t"] = np.float32(1e30)
    hits_o, t_o, _, _ = O.Oracle(sc).trace_closest(1, rays)
    c = S.Compute().Init()
    try:
        c.bind_scene(sc)
        c.SetUInt("bvh_count", 1)
        hits, t = c.trace_closest(rays)
    finally:
        c.close()
    assert (hits == hits_o).all() and bits_equal(t, t_o).all()
    hit = hits != 0xFFFFFFFF
    assert hit.mean() > 0.95
    # a hit on a red or green triangle is a tie by construction (its twin computes the same t bit for bit)
    twins = _twin_index(sc)
    assert (twins[hits[hit]] >= 0).mean() > 0.3


def _twin_index(sc):
    """Per triangle, the index of the other triangle with the same three corners (-1 if none)."""
    corners = sc.verts["pos"][sc.tris["v"]].reshape(len(sc.tris), 9)
    out = np.full(len(sc.tris), -1, np.int64)
    seen = {}
    for i, row in enumerate(corners):
        k = row.tobytes()
        if k in seen:
            out[i], out[seen[k]] = seen[k], i
        else:
            seen[k] = i
    return out


def test_textured_material_albedo(tmp_path):
    import test_producers as P

    w, h = 4, 4
    px = [200, 100, 50] * (w * h)
    P._write_png(tmp_path / "t.png", w, h, px)
    (tmp_path / "m.mtl").write_text("newmtl tex\nKd 1 1 1\nKs 0.3 0.3 0.3\nNs 30\nmap_Kd t.png\n")
    verts = "v -6 0 -6\nv 6 0 -6\nv 6 12 -6\nv -6 12 -6\n"
    (tmp_path / "m.obj").write_text("mtllib m.mtl\n" + verts + "usemtl tex\nf 1 2 3 4\n")
    setup = R.make_setup(32, 32, show_model=True, models=[S.load_obj(tmp_path / "m.obj")])
    assert_parity(setup, 2)


def _textured_obj(tmp_path):
    """Two textured quads (RGB and single-channel PNGs) whose vt coordinates leave [0,1], so REPEAT wraps."""
    import test_producers as P

    rng = np.random.default_rng(7)
    P._write_png(tmp_path / "a.png", 8, 6, [int(x) for x in rng.integers(0, 256, 8 * 6 * 3)])
    P._write_png(tmp_path / "b.png", 5, 3, [int(x) for x in rng.integers(0, 256, 5 * 3)], ctype=0)
    (tmp_path / "m.mtl").write_text("newmtl a\nKd 1 1 1\nKs 0.3 0.3 0.3\nNs 30\nmap_Kd a.png\n"
                                    "newmtl b\nKd 1 1 1\nKs 0.1 0.1 0.1\nNs 5\nmap_Kd b.png\n")
    (tmp_path / "m.obj").write_text(
        "mtllib m.mtl\n"
        "v -20 -2 -6\nv 20 -2 -6\nv 20 28 -6\nv -20 28 -6\nv -20 -2 25\nv 20 -2 25\n"
        "vt -1.3 -0.7\nvt 2.6 -0.7\nvt 2.6 2.7\nvt -1.3 2.7\nvt 0.25 3.5\nvt 4.75 3.5\n"
        "usemtl a\nf 1/1 2/2 3/3 4/4\n"
        "usemtl b\nf 5/5 6/6 2/2 1/1\n")
    return tmp_path / "m.obj"


def test_sampled_texture_parity(tmp_path):
    """textures sampled at the hit's interpolated uv (loader with has_texcoords set)."""
    setup = R.make_setup(48, 40, show_model=True, models=[S.load_obj(_textured_obj(tmp_path), texcoords=True)])
    assert setup.scene.sample_textures and len(setup.scene.textures) == 2
    assert_parity(setup, 3)


def test_sampled_texture_at_zero_uv_is_the_constant_albedo(tmp_path):
    """With the reference's loader every uv is (0,0): sampling per hit gives the precomputed tex_albedo, bit for bit."""
    import dataclasses

    setup = R.make_setup(48, 40, show_model=True, models=[S.load_obj(_textured_obj(tmp_path))])
    assert not setup.scene.sample_textures
    a, o, _ = gpu_render(setup, 3)
    sampled = dataclasses.replace(setup, scene=dataclasses.replace(setup.scene, sample_textures=True))
    b, p, _ = gpu_render(sampled, 3)
    assert bits_equal(a, b).all() and (o == p).all()


def test_sampled_texture_two_models_with_transform(tmp_path):
    """The hit's model-space point comes from the frame of the BVH that owns the triangle; a ghost record
    (bvh_count beyond the models) never hits."""
    obj = _textured_obj(tmp_path)
    setup = R.make_setup(48, 40, show_model=True, models=[S.load_obj(obj, texcoords=True),
                                                          S.load_obj(obj, texcoords=True)], bvh_count=3)
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (4.0, -3.0, 7.0)
    setup.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(setup, 2)


def test_synthetic_mesh_global_mode():
    """A 30k-triangle mesh: too big for the LDS copy, exercises the global-memory traversal."""
    setup = R.make_setup(40, 30, show_model=True, models=[R.synthetic_model(30000, seed=3)])
    assert_parity(setup, 2)


def test_surface_mesh_global_mode():
    """bench.py's surface_mesh leg: the 262k-triangle torus-knot tube (global-scene mode) against the oracle."""
    setup = R.make_setup(64, 40, show_model=True, models=[R.torus_knot_model()])
    assert_parity(setup, 2)


@pytest.mark.parametrize("env", [{"SRT_NODE_ALIGN": "1"}, {"SRT_NODE_LAYOUT": "0"},
                                 {"SRT_NODE_ALIGN": "1", "SRT_GLOBAL_FUSED_MODE": "1"},
                                 {"SRT_NODE_ALIGN": "0", "SRT_GLOBAL_FUSED_MODE": "0"},
                                 {"SRT_NODE_LAYOUT": "0", "SRT_GLOBAL_FUSED_MODE": "1"},
                                 {"SRT_GLOBAL_WAVES_MODE": "4"},
                                 {"SRT_NODE_ALIGN": "1", "SRT_GLOBAL_WAVES_MODE": "5"}])
def test_node_layouts_global_mode(monkeypatch, env):
    """The device node layouts (pathtrace.hip LayoutNodes): line-aligned right-child chains (chosen for
    scenes past the Infinity Cache) and the reference's own order (no right-spine double steps) render
    the oracle's frame in global-scene mode, two models with a moved second one included; so do both
    traversal schedules (fused sub-steps, chosen with the dense layout, and the IL pattern) on
    every layout, and the fused schedule's timed instance at 4 and 5 waves per SIMD (8-entry LDS
    rings: deeper stacks spill to HBM more often)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    setup = R.make_setup(48, 40, show_model=True, models=[R.synthetic_model(30000, seed=3)])
    assert_parity(setup, 2)
    two = R.make_setup(40, 32, show_model=True, models=[R.synthetic_model(20000, seed=4),
                                                        R.synthetic_model(5000, seed=6)])
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (1.5, -2.0, 0.5)
    two.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(two, 2)


@pytest.mark.parametrize("env", [{"SRT_TRI_ALIGN": "1", "SRT_NODE_ALIGN": "1", "SRT_GLOBAL_FUSED_MODE": "0"},
                                 {"SRT_TRI_ALIGN": "1", "SRT_GLOBAL_FUSED_MODE": "1"},
                                 {"SRT_TRI_ALIGN": "1", "SRT_NODE_LAYOUT": "0", "SRT_GLOBAL_FUSED_MODE": "0"},
                                 {"SRT_TRI_ALIGN": "1"},
                                 {"SRT_TRI_ALIGN": "0", "SRT_GLOBAL_FUSED_MODE": "0"}])
def test_triangle_slots(monkeypatch, tmp_path, rubik, env):
    """Line-aligned triangle slots (pathtrace.hip LayoutTris, chosen for every scene of 1 MB or more):
    gaps of zero records between small leaves, leaf and BVH triangle ranges remapped.  Global mode on
    both schedules and the LDS kernel (Rubik, forced) render the oracle's frame; a moved second model and
    sampled textures (the hit's BVH found by its slot range) too; the closest-hit query returns input
    triangle indices.  The identity layout (forced) is checked the same way."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    soup = R.make_setup(48, 40, show_model=True, models=[R.synthetic_model(30000, seed=3)])
    r = R.Renderer(soup)
    try:
        slots = r.compute.GetInt("scene.tri_slots")
        # the soup's 1- and 2-triangle leaves leave gaps
        assert slots == 30000 if env["SRT_TRI_ALIGN"] == "0" else slots > 30000
    finally:
        r.close()
    assert_parity(soup, 2)
    two = R.make_setup(40, 32, show_model=True, models=[R.synthetic_model(20000, seed=4),
                                                        R.synthetic_model(5000, seed=6)])
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (1.5, -2.0, 0.5)
    two.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(two, 2)
    obj = _textured_obj(tmp_path)
    tex = R.make_setup(48, 40, show_model=True, models=[S.load_obj(obj, texcoords=True),
                                                        S.load_obj(obj, texcoords=True)], bvh_count=3)
    tex.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(tex, 2)
    assert_parity(R.make_setup(64, 48, show_model=True, models=[rubik]), 2)
    for scene, n in ((S.Scene.from_models([rubik]), 20000), (soup.scene, 4000)):
        rays = _kat_rays(n, 11)
        hits_o, t_o, _, _ = O.Oracle(scene).trace_closest(1, rays)
        c = S.Compute().Init()
        try:
            c.bind_scene(scene)
            c.SetUInt("bvh_count", 1)
            hits, t = c.trace_closest(rays)
        finally:
            c.close()
        assert (hits == hits_o).all() and bits_equal(t, t_o).all()


@pytest.mark.parametrize("depth", [None, "3", "1", "0", "14"])
def test_top_levels_in_lds(monkeypatch, depth):
    """The fused global-scene instance's LDS copy of the tree's top levels (pathtrace.hip LayoutNodes lays
    their pairs out first; traversal.hpp trav_fused reads them from LDS): as deep as fits by default, or
    SRT_TOP_DEPTH levels, or none; one and two BVHs (a moved second model) render the oracle's frame, and
    the timed (fused) instance equals the counting one bit for bit (gpu_render)."""
    if depth is not None:
        monkeypatch.setenv("SRT_TOP_DEPTH", depth)
    soup = R.make_setup(48, 40, show_model=True, models=[R.synthetic_model(30000, seed=3)])
    r = R.Renderer(soup)
    try:
        want = {None: None, "3": 3, "1": 1, "0": 0, "14": 14}[depth]
        got = r.compute.GetInt("scene.top_depth")
        assert r.compute.GetInt("scene.fused") == 1
        assert got == want if want is not None else got >= 6
        r.render(1)
        r.finish()
        top_f4 = r.compute.GetInt("launch.top_f4")
        if depth == "14":  # a forced region past the LDS a block may take: laid out, not copied
            assert r.compute.GetInt("scene.top_f4") > 0 and top_f4 == 0
        else:
            assert top_f4 == r.compute.GetInt("scene.top_f4") and (top_f4 > 0) == (got > 0)
    finally:
        r.close()
    assert_parity(soup, 2)
    two = R.make_setup(40, 32, show_model=True, models=[R.synthetic_model(20000, seed=4),
                                                        R.synthetic_model(5000, seed=6)])
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (1.5, -2.0, 0.5)
    two.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(two, 2)


def test_launch_occupancy_reported(rubik):
    """srt_get_int's launch.block / launch.blocks_per_cu report each kernel's resident occupancy: the LDS
    kernel one 1024-lane block per CU (4 waves per SIMD), the fused global instance of a small tree five
    256-lane blocks (5 waves), of a 1 M-triangle soup four (4 waves), the sphere kernel five."""
    cases = [(R.make_setup(32, 24, show_model=True, models=[rubik]), 1024, 1),
             (R.make_setup(32, 24, show_model=True, models=[R.torus_knot_model()]), 256, 5),
             (R.make_setup(32, 24, show_model=True, models=[R.synthetic_model(1_000_000)]), 256, 4),
             (R.make_setup(32, 24, show_model=False), 256, 5)]
    for setup, block, per_cu in cases:
        r = R.Renderer(setup)
        try:
            r.render(1)
            r.finish()
            got = (r.compute.GetInt("launch.block"), r.compute.GetInt("launch.blocks_per_cu"))
        finally:
            r.close()
        assert got == (block, per_cu), (got, block, per_cu)


@pytest.mark.parametrize("n_mats,mats_in_lds", [(1, True), (100, True), (150, True), (175, False), (200, False),
                                                (600, False)])
def test_top_region_keeps_occupancy_with_many_materials(n_mats, mats_in_lds):
    """the top levels' LDS region is sized beside the rings and the launch's light records, and
    the material records (placed behind it in the same block's LDS) only go there when they still fit the
    block's share, so many materials never cost the 5-wave fused instance a resident block per CU, and never
    its region either: the knot (5 waves per SIMD, 256-lane blocks) keeps 5 blocks per CU and its 7-level
    region with 1 to 600 materials; up to 150 (4.8 KB of records) sit in LDS beside the 16-KB rings, the
    10-KB region and the lights, 175, 200 and 600 are read from HBM (5.6 KB: past the block's 32,000-B share,
    though inside the 32,768 B the occupancy API accepts for 5 blocks -- gfx950 allocates LDS in 1,280-B
    units, tools/probes/lds_fit.hip; 6.4 KB; 19.2 KB: also past the 16-KB LDS cap); the frame matches the
    oracle."""
    import dataclasses

    base = R.make_setup(48, 40, show_model=True, models=[R.torus_knot_model()])
    sc = base.scene
    mats = np.resize(sc.mats, n_mats).copy()
    mats["diffuse"] = np.stack([np.linspace(0.2, 0.9, n_mats), np.linspace(0.9, 0.3, n_mats),
                                np.full(n_mats, 0.5)], axis=1).astype(np.float32)
    tris = sc.tris.copy()
    tris["mat"] = np.arange(len(tris), dtype=np.uint32) % n_mats
    scene = dataclasses.replace(sc, mats=mats, tex_albedo=np.resize(sc.tex_albedo, (n_mats, 3)).copy(), tris=tris)
    setup = dataclasses.replace(base, scene=scene)
    r = R.Renderer(setup)
    try:
        c = r.compute
        assert c.GetInt("scene.fused") == 1 and c.GetInt("scene.global_waves") == 5
        r.render(1)
        r.finish()
        assert c.GetInt("launch.block") == 256 and c.GetInt("launch.blocks_per_cu") == 5
        assert c.GetInt("launch.top_f4") == c.GetInt("scene.top_f4") > 0 and c.GetInt("scene.top_depth") >= 7
        assert c.GetInt("launch.mats_lds") == int(mats_in_lds)
    finally:
        r.close()
    assert_parity(setup, 2)


@pytest.mark.parametrize("case", ["overlap", "shared"])
def test_triangle_slots_unusual_leaves(case):
    """LayoutTris on leaf ranges no reference-built tree has: a leaf grown by one triangle into the next
    leaf's range (partly overlapping ranges: the identity layout is kept) and a leaf given another leaf's
    range (the same range twice: slotted once).  Both render the oracle's frame."""
    import dataclasses

    setup = R.make_setup(48, 40, show_model=True, models=[R.synthetic_model(30000, seed=3)])
    n = setup.scene.nodes.copy()
    leaves = np.flatnonzero(n["count"] > 0)
    starts = {int(n["first"][i]): i for i in leaves}
    i = next(i for i in leaves if int(n["first"][i] + n["count"][i]) in starts)
    if case == "overlap":
        n["count"][i] += 1
    else:
        j = starts[int(n["first"][i] + n["count"][i])]
        n["first"][j], n["count"][j] = n["first"][i], n["count"][i]
    mod = dataclasses.replace(setup, scene=dataclasses.replace(setup.scene, nodes=n))
    r = R.Renderer(mod)
    try:
        slots = r.compute.GetInt("scene.tri_slots")
    finally:
        r.close()
    assert slots == 30000 if case == "overlap" else slots > 30000
    assert_parity(mod, 2)


@pytest.mark.parametrize("layout", ["1", "0"])
def test_unreachable_garbage_nodes(monkeypatch, layout):
    """Records no traversal reaches may hold anything: a leaf whose triangle range lies far past
    the array and an internal node whose children do, appended to a soup's node array.  The upload checks
    and lays out (triangle slots forced on; node layout laid out or kept) only the nodes reachable from
    the BVH roots and node 0, and the frame is the oracle's."""
    import dataclasses

    monkeypatch.setenv("SRT_TRI_ALIGN", "1")
    monkeypatch.setenv("SRT_NODE_LAYOUT", layout)
    setup = R.make_setup(48, 40, show_model=True, models=[R.synthetic_model(30000, seed=3)])
    n = setup.scene.nodes
    m = np.zeros(len(n) + 2, dtype=n.dtype)
    m[:len(n)] = n
    m["first"][-2], m["count"][-2] = 0xFFFFFF00, 5     # a leaf past the triangles
    m["first"][-1], m["count"][-1] = 0xFFFFFFF0, 0     # an internal node past the nodes
    mod = dataclasses.replace(setup, scene=dataclasses.replace(setup.scene, nodes=m))
    r = R.Renderer(mod)
    try:
        assert r.compute.GetInt("scene.tri_slots") > 30000
    finally:
        r.close()
    assert_parity(mod, 2)


def test_global_schedule_chosen_by_scene_size():
    """srt_upload_scene's choices for the timed global-scene instance, as bench.py reports them: the torus
    knot (20 MB of nodes + triangles) takes fused sub-steps at 5 waves per SIMD, a 1 M soup (101 MB)
    fused sub-steps at 4; the environment forces either."""
    def chosen(model, env=None):
        old = {k: os.environ.get(k) for k in (env or {})}
        os.environ.update(env or {})
        try:
            r = R.Renderer(R.make_setup(16, 8, show_model=True, models=[model]))
            try:
                return r.compute.GetInt("scene.fused"), r.compute.GetInt("scene.global_waves")
            finally:
                r.close()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v

    knot = R.torus_knot_model()
    assert chosen(knot) == (1, 5)
    assert chosen(knot, {"SRT_GLOBAL_WAVES_MODE": "4"}) == (1, 4)
    assert chosen(R.synthetic_model(1_000_000, seed=1)) == (1, 4)


@pytest.mark.parametrize("force_global", ["1", "0"])
def test_bvh_records_sharing_a_subtree(rubik, monkeypatch, force_global):
    """Two BVH records whose trees share subtrees: the second record's root is a new node
    whose child pair copies the first tree's root children, child indices included, so both trees reach
    the same grandchild pairs.  The device layout places a shared pair once, under the first tree; the
    second tree's new pair is laid elsewhere, so its node must not claim that its right child's pair
    follows it (the global-mode right-spine step would read the wrong pair).  The second record is
    moved so both trees are hit."""
    import dataclasses

    monkeypatch.setenv("SRT_FORCE_GLOBAL_SCENE", force_global)
    setup = R.make_setup(48, 40, show_model=True, models=[rubik])
    n = setup.scene.nodes
    L = len(n)
    c0 = int(n[0]["first"])
    assert n[0]["count"] == 0 and n[c0 + 1]["count"] == 0  # the root's right child is internal
    m = np.concatenate([n, np.zeros(3, n.dtype)])
    m[L] = n[0]
    m[L]["first"] = L + 1
    m[L + 1], m[L + 2] = n[c0], n[c0 + 1]  # copies: their children are the first tree's pairs
    bvhs = np.concatenate([setup.scene.bvhs, setup.scene.bvhs[:1]])
    bvhs[1]["first_index"] = L
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (7.0, -1.0, -3.0)
    bvhs[1]["frame"] = frame.reshape(16)
    shared = dataclasses.replace(setup, scene=dataclasses.replace(setup.scene, nodes=m, bvhs=bvhs), bvh_count=2)
    assert_parity(shared, 2)


@pytest.mark.parametrize("layout", ["1", "0"])
def test_lds_mode_node_orders(rubik, monkeypatch, layout):
    """LDS mode reads node pairs from 80-B blocks (traversal.hpp node_pair) in both device orders: the
    traversal-order layout and the reference's own order (SRT_NODE_LAYOUT=0, no child-index flags)."""
    monkeypatch.setenv("SRT_NODE_LAYOUT", layout)
    assert_parity(R.make_setup(56, 40, show_model=True, models=[rubik]), 2)


@pytest.mark.parametrize("layout", ["1", "0"])
def test_overlapping_sibling_pairs(rubik, monkeypatch, layout):
    """A node array whose child pairs start at even slots (a zero node inserted after the root shifts every
    pair by one).  Laid out again it takes LDS mode; kept in its own order (SRT_NODE_LAYOUT=0) its pairs are
    not 64-B blocks, so the scene is traversed in global-scene mode.  Both render the oracle's frame."""
    import dataclasses

    monkeypatch.setenv("SRT_NODE_LAYOUT", layout)
    setup = R.make_setup(48, 40, show_model=True, models=[rubik])
    n = setup.scene.nodes
    m = np.zeros(len(n) + 1, dtype=n.dtype)
    m[0] = n[0]
    m[2:] = n[1:]
    internal = m["count"] == 0
    internal[1] = False  # the inserted zero record is unreachable
    m["first"][internal] += 1
    assert (m["first"][internal] % 2 == 0).all()
    bvhs = setup.scene.bvhs.copy()
    assert (bvhs["first_index"] == 0).all()
    shifted = dataclasses.replace(setup, scene=dataclasses.replace(setup.scene, nodes=m, bvhs=bvhs))
    a, o = assert_parity(shifted, 2)
    b, p, _ = gpu_render(setup, 2)
    assert bits_equal(a, b).all() and (o == p).all()


@pytest.mark.parametrize("n_tris", [600, 700])
def test_lds_budget_boundary(n_tris):
    """Meshes on either side of the LDS budget: 600 triangles (depth 11) is the fullest LDS-resident copy,
    nodes at the 80-B pair stride + triangles + 1024 lanes' stacks = 157,248 of 163,840 bytes; 700 (depth 12)
    no longer fits and is traversed in global-scene mode.  Both render the oracle's frame."""
    setup = R.make_setup(48, 40, show_model=True, models=[R.synthetic_model(n_tris, seed=5)])
    assert_parity(setup, 2)


def test_lds_and_global_modes_agree(rubik, monkeypatch):
    setup = R.make_setup(64, 48, show_model=True, models=[rubik])
    a, o, _ = gpu_render(setup, 3)
    monkeypatch.setenv("SRT_FORCE_GLOBAL_SCENE", "1")
    b, p, _ = gpu_render(setup, 3)
    assert bits_equal(a, b).all() and (o == p).all()


def test_sample_buffer_chunking_invariance(rubik, monkeypatch):
    setup = R.make_setup(64, 48, show_model=True, models=[rubik])
    a, o, _ = gpu_render(setup, 9)
    monkeypatch.setenv("SRT_SAMPLE_BUFFER_KB", "100")  # 2 frames of 64x48 per chunk -> 5 chunks
    b, p, _ = gpu_render(setup, 9)
    assert bits_equal(a, b).all() and (o == p).all()


def test_schedule_invariance(rubik, monkeypatch):
    """The work schedule decides which wave traces which sample, never a value: the tile order learned
    from the previous launch, the natural order, and single-batch claims everywhere or nowhere give the
    same bits."""
    setup = R.make_setup(72, 56, show_model=True, models=[rubik])
    r = R.Renderer(setup)
    try:
        r.render(4, count=True)  # records the tile costs
        r.render(4)              # runs in the learned order
        r.finish()
        a, o = r.accum(), r.output()
    finally:
        r.close()
    for env in ({"SRT_TILE_ORDER": "0"}, {"SRT_TAIL_CLAIMS": "0"}, {"SRT_TAIL_CLAIMS": "100000"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        b, p, _ = gpu_render(setup, 4)
        assert bits_equal(a, b).all() and (o == p).all(), env
        for k in env:
            monkeypatch.delenv(k)


def test_global_schedule_invariance(monkeypatch):
    """The same for the fused 5-wave global-scene instance, whose tail window is its own (8 claims per
    wave, pathtrace.hip tail_claims_gw5): the default window, none, 16 claims and the whole launch give
    the same bits, and the default renders the oracle's frame.  At this size every window covers the
    whole launch but 0; the window's edge inside a launch is crossed by the at-size C3 stand-in tests
    (test_gpu_configs.py), whose timed instance is this one."""
    setup = R.make_setup(64, 48, show_model=True, models=[R.synthetic_model(30000, seed=3)])
    r = R.Renderer(setup)
    try:
        assert r.compute.GetInt("scene.fused") == 1 and r.compute.GetInt("scene.global_waves") == 5
    finally:
        r.close()
    a, o, _ = gpu_render(setup, 3)
    for v in ("0", "16", "100000"):
        monkeypatch.setenv("SRT_TAIL_CLAIMS", v)
        b, p, _ = gpu_render(setup, 3)
        assert bits_equal(a, b).all() and (o == p).all(), v
    monkeypatch.delenv("SRT_TAIL_CLAIMS")
    assert_parity(setup, 3)


@pytest.mark.parametrize("nranks,band", [(2, 16), (3, 8), (2, 2), (3, 3), (8, 2), (5, 1)])
def test_row_band_tiling_reassembles(rubik, nranks, band):
    import torch

    W, H = 64, 56
    setup = R.make_setup(W, H, show_model=True, models=[rubik])
    full, full_out, _ = gpu_render(setup, 3)
    nb = (H + band - 1) // band
    rows_pad = ((nb + nranks - 1) // nranks) * band
    gathered = torch.zeros((nranks, rows_pad, W, 4), dtype=torch.float32, device="cuda")
    for rank in range(nranks):
        loc, _, _ = gpu_render(setup, 3, rank=rank, nranks=nranks, band_rows=band)
        gathered[rank, :loc.shape[0]] = torch.from_numpy(loc).cuda()
    torch.cuda.synchronize()
    r = R.Renderer(setup)
    try:
        acc = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        out = torch.empty((H, W), dtype=torch.int32, device="cuda")
        r.compute.assemble_bands(gathered.data_ptr(), nranks, rows_pad, band, 4, acc.data_ptr(), out.data_ptr())
        r.finish()
        torch.cuda.synchronize()
    finally:
        r.close()
    assert bits_equal(acc.cpu().numpy(), full).all()
    assert (out.cpu().numpy().view(np.uint8).reshape(H, W, 4) == full_out).all()


def _kat_rays(n, seed):
    rng = np.random.default_rng(seed)
    rays = np.zeros(n, S.RAY_DTYPE)
    rays["o"] = rng.uniform([-15, -3, -15], [15, 22, 15], size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[::7, 0] = 0.0          # zero components: infinite 1/d in the slab test
    d[::11, 1:] = 0.0
    d[5] = 0.0               # the zero direction
    rays["d"] = d
    rays["t"] = np.where(np.arange(n) % 5 == 0, np.float32(3.0), np.float32(1e30))
    rays[0]["o"], rays[0]["d"] = (-10.0, 3.0, 6.0), np.array([0.9838, -0.0118, 0.1787], np.float32)
    rays[1]["o"], rays[1]["d"] = (0.0, 0.0, 0.0), (0.0, 1.0, 0.0)
    return rays


def test_trace_closest_matches_oracle(rubik):
    scene = S.Scene.from_models([rubik])
    rays = _kat_rays(20000, 11)
    hits_o, t_o, _, st = O.Oracle(scene).trace_closest(1, rays)
    c = S.Compute().Init()
    try:
        c.bind_scene(scene)
        c.SetUInt("bvh_count", 1)
        hits, t = c.trace_closest(rays)
    finally:
        c.close()
    assert hits[0] == 365 and hits[1] != 0xFFFFFFFF
    assert (hits == hits_o).all()
    assert bits_equal(t, t_o).all()
    assert (hits != 0xFFFFFFFF).sum() > 1000


def test_reference_kat_through_trace_closest(rubik):
    """The reference's own GL integration test (BVH_intergration_tests.cpp:63-113) through srt_trace_closest,
    as a maintainer would bind it: 64 rays, bvh_count 1.  Every odd ray hits the loader's triangle 17, the
    reference's expected value (:94), reported in BVH order (365) as the shader's Intersects does and mapped
    back through srt_scene_tri_order.  The even rays hit loader triangle 176 at t = 5.9054995 where :94 expects a
    miss (test_oracle_pins.py: every reading tried still hits; an unexplained disagreement).  After
    UpdateModelMatrix(0, mat4(1e-6) with [c][3] set) every ray misses (:96-113)."""
    from test_oracle_pins import kat_rays

    scene = S.Scene.from_models([rubik])
    rays = kat_rays(64)
    c = S.Compute().Init()
    try:
        c.bind_scene(scene)
        c.SetUInt("bvh_count", 1)
        hits, t = c.trace_closest(rays)
        assert (hits[1::2] == 365).all() and (scene.tri_input[hits[1::2]] == 17).all()
        assert (scene.tri_input[hits[0::2]] == 176).all()
        hits_o, t_o, _, _ = O.Oracle(scene).trace_closest(1, rays)
        assert (hits == hits_o).all() and bits_equal(t, t_o).all()
        m = np.zeros((4, 4), np.float32)
        for i in range(4):
            m[i, i] = 0.000001
        m[0, 3], m[1, 3], m[2, 3] = 10, 1000, 10
        S.UpdateModelMatrix(c, 0, m)
        hits, _ = c.trace_closest(rays)
        assert (hits == 0xFFFFFFFF).all()
    finally:
        c.close()


def test_full_frame_rows_and_determinism(rubik):
    """BASELINE frame size (1920x1080): oracle rows sampled across the frame, bit-exact; two runs identical."""
    W, H, spp = 1920, 1080, 2
    setup = R.make_setup(W, H, show_model=True, models=[rubik])
    a, o, st = gpu_render(setup, spp)
    rows = np.arange(3, H, 97, dtype=np.int32)
    acc, out, _ = oracle_render(setup, spp, rows=rows)
    assert bits_equal(a[rows], acc[rows]).all()
    assert (o[rows] == out[rows]).all()
    b, p, st2 = gpu_render(setup, spp)
    assert bits_equal(a, b).all() and (o == p).all() and st["rays"] == st2["rays"]
    assert np.isfinite(a[..., :3]).mean() > 0.999 and (a[..., 3] == 1.0).all()


def test_cpp_api_program(rubik, tmp_path):
    """The C++ mirror API running the reference's integration test + main loop (tests/cpp/test_api.cpp);
    the loop's frame (a scripted camera move resets it: reset + 3 sampled frames of Rubik at 64x48 from the
    moved camera) is checked against the oracle."""
    exe = ROOT / "tests" / "cpp" / "_build" / "test_api"
    exe.parent.mkdir(exist_ok=True)
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", str(ROOT / "include"), str(ROOT / "tests/cpp/test_api.cpp"),
                    "-o", str(exe), "-L", str(PKG), "-lsrt_amd", f"-Wl,-rpath,{PKG}"], check=True)
    shaders = tmp_path / "shaders"
    shaders.mkdir()
    for name in ("raytrace_compute.glsl", "ray_intersects.glsl"):  # CreateComputeProgram opens the file
        (shaders / name).write_text("#version 450\n")
    res = subprocess.run([str(exe), str(OBJECTS) + "/", str(shaders) + "/", str(tmp_path / "loop")],
                         capture_output=True, text=True, timeout=120)
    assert res.returncode == 0 and res.stdout.startswith("OK"), res.stdout + res.stderr
    acc = np.fromfile(tmp_path / "loop.accum", np.float32).reshape(48, 64, 4)
    out = np.fromfile(tmp_path / "loop.rgba8", np.uint8).reshape(48, 64, 4)
    from oracle import scene_ref as REF

    setup = R.make_setup(64, 48, show_model=True, models=[rubik])
    cam = REF.CameraRef(True)  # test_api.cpp's script: 3 idle frames, then W + a (10, -5) drag for 0.5 s
    for frame in range(4):
        drag = frame == 3
        REF.progressive_frame_ref(cam, (0.0, 0.0, 1.0 if drag else 0.0), (10.0, -5.0) if drag else (0.0, 0.0),
                                  drag, frame == 0, 0.5, 0)
    setup.camera = cam
    want_acc, want_out, _ = oracle_render(setup, 3)
    assert bits_equal(acc, want_acc).all()
    assert (out == want_out).all()


def test_save_image_matches_output(rubik, tmp_path):
    """Output stage on a rendered frame: the PNG holds image0's bytes, top row first."""
    from test_output_stage import _read_png

    setup = R.make_setup(48, 40, show_model=True, models=[rubik])
    r = R.Renderer(setup)
    try:
        r.render(2)
        r.finish()
        out = r.output()
        r.compute.save_image(tmp_path / "frame.png")
    finally:
        r.close()
    assert (_read_png(tmp_path / "frame.png") == out[::-1]).all()


@pytest.mark.parametrize("yaw,pitch,origin", [(25.0, -12.0, (3.0, 12.0, 30.0)), (-70.0, 40.0, (-14.0, 6.0, 14.0)),
                                              (180.0, -89.0, (0.5, 25.0, 0.25)), (40.0, 10.0, (0.3, 4.0, 0.7))])
def test_moved_camera_parity(rubik, yaw, pitch, origin):
    """Camera::Rotate / a moved origin (the reference's interactive path, camera.cpp:107-212): rays leave the
    cube at grazing and inside-out angles, through the box faces the default camera never sees; the last
    camera sits inside the model's bounds, among the cubies, so every camera ray starts inside the root box
    and IntersectsBox answers with its exit distance (ray_intersects.glsl:57), which then culls by it."""
    setup = R.make_setup(48, 40, show_model=True, models=[rubik])
    setup.camera.Rotate(yaw, pitch)
    setup.camera.position = np.asarray(origin, np.float32)
    assert_parity(setup, 2)


@pytest.mark.parametrize("mode", ["lds", "global"])
def test_pathological_triangles(monkeypatch, mode):
    """Triangles no exporter should write, inside a floor the camera sees: zero-area (collinear corners), a
    point, a sliver 1e-6 wide, corners at +-1e30 (infinite edges and products in IntersectsTriangle), one
    NaN corner (NaN bounds up the tree: the slab test's IEEE minNum/maxNum decide) and a huge triangle
    spanning the scene.  The builder, both scene modes and the shading all take them; the frame is the
    oracle's."""
    if mode == "global":
        monkeypatch.setenv("SRT_FORCE_GLOBAL_SCENE", "1")
    rng = np.random.default_rng(41)
    quads = []
    for i in range(6):
        for j in range(6):
            x0, z0 = -12 + 4 * i, -12 + 4 * j
            quads += [[x0, 0, z0, x0 + 4, 0, z0, x0 + 4, 0, z0 + 4], [x0, 0, z0, x0 + 4, 0, z0 + 4, x0, 0, z0 + 4]]
    bad = [[-2, 3, -2, 0, 4, -1, 2, 5, 0],                     # collinear: zero area
           [1, 6, 1, 1, 6, 1, 1, 6, 1],                        # a point
           [-3, 2, 3, 3, 2, 3, 0, 2 + 1e-6, 3],                # a sliver
           [0, 8, -4, 1e30, 8, -4, 0, 8, 1e30],                # infinite edges
           [-1e30, 9, 0, 2, 9, 0, 0, -1e30, 1],
           [4, 3, 4, 5, float("nan"), 4, 4, 4, 5],             # a NaN corner
           [-40, 12, -40, 40, 14, -40, 0, 13, 40]]             # spans everything
    bumps = rng.uniform(-8, 8, (40, 9)).astype(np.float32)
    bumps[:, 1::3] = np.abs(bumps[:, 1::3]) * 0.5 + 1.0
    xyz = np.concatenate([np.asarray(quads, np.float32), np.asarray(bad, np.float32), bumps])
    model = S.model_from_triangles(xyz, kd=(0.7, 0.6, 0.5), ks=(0.3, 0.3, 0.3), ns=40.0)
    setup = R.make_setup(48, 40, show_model=True, models=[model])
    assert_parity(setup, 2)


def test_moved_camera_spheres_parity():
    setup = R.make_setup(40, 48, show_model=False)
    setup.camera.Rotate(-35.0, 20.0)
    setup.camera.position = np.asarray((1.5, 0.5, 2.0), np.float32)
    assert_parity(setup, 3)


def test_reference_upload_path_renders_oracle_frame(rubik, tmp_path):
    """tests/cpp/test_ref_loader.cpp render: gpu_loader.cpp's own flattening handed to srt_upload_scene
    (two Rubik models, the second moved by UpdateModelMatrix, bvh_count 2) renders the frame that
    srt_upload_scene_obj renders, and that frame is the oracle's."""
    from test_boundary import _build

    exe = _build("test_ref_loader")
    res = subprocess.run([str(exe), "render", str(OBJECTS) + "/", str(tmp_path / "ref")], capture_output=True,
                         text=True, timeout=120)
    assert res.returncode == 0 and res.stdout.startswith("OK render"), res.stdout + res.stderr
    acc = np.fromfile(tmp_path / "ref.accum", np.float32).reshape(48, 64, 4)
    setup = R.make_setup(64, 48, show_model=True, models=[rubik, S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")])
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (12.0, -2.0, -5.0)
    setup.scene.bvhs[1]["frame"] = frame.reshape(16)
    want, _, _ = oracle_render(setup, 3)
    assert bits_equal(acc, want).all()


# ---- pool_kernel (pool.hpp, SRT_POOL=1): LDS mode with workgroup ray pools ----
@pytest.mark.parametrize("w,h,spp,depth", [(64, 64, 2, 5), (96, 54, 4, 5), (31, 23, 3, 8), (40, 72, 2, 0)])
def test_pool_kernel_parity(rubik, monkeypatch, w, h, spp, depth):
    """The pool kernel (hits shaded by shading waves from LDS records) renders the oracle's frame, with
    the counting instance's CheckHit counts, in the fused and the per-frame dispatch paths."""
    monkeypatch.setenv("SRT_POOL", "1")
    monkeypatch.setenv("SRT_POOL_DEADLINE_MS", "20000")
    setup = R.make_setup(w, h, show_model=True, models=[rubik], max_depth=depth)
    assert_parity(setup, spp)
    assert_parity(setup, spp, per_frame=True)


def test_pool_kernel_scenes_and_tiling(rubik, monkeypatch):
    """Pool mode on two models with a moved second one (BVH switches inside traversal lanes), a
    multi-rank band split and small pool batches / record counts: every frame is the oracle's."""
    monkeypatch.setenv("SRT_POOL", "1")
    monkeypatch.setenv("SRT_POOL_DEADLINE_MS", "20000")
    second = S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")
    two = R.make_setup(48, 40, show_model=True, models=[rubik, second])
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (12.0, -2.0, -5.0)
    two.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(two, 2)
    monkeypatch.setenv("SRT_POOL_BATCH", "8")
    monkeypatch.setenv("SRT_POOL_SLOTS", "64")
    setup = R.make_setup(64, 48, show_model=True, models=[rubik])
    acc, out = assert_parity(setup, 3)
    parts = [gpu_render(setup, 3, rank=r, nranks=3, band_rows=8)[0] for r in range(3)]
    from srt_amd import parallel as PAR

    rows_pad = PAR.rows_pad(48, 8, 3)
    stacked = np.zeros((3, rows_pad, 64, 4), np.float32)
    for r, p in enumerate(parts):
        stacked[r, :len(p)] = p
    assert bits_equal(PAR.assemble_host(stacked, 48, 8), acc).all()


def test_pool_kernel_metric_frame_equals_sample_kernel(rubik, monkeypatch):
    """The metric frame (1920x1080) at 16 spp: pool mode's accumulation and image equal sample_kernel's."""
    setup = R.make_setup(1920, 1080, show_model=True, models=[rubik])
    a, o, st = gpu_render(setup, 16)
    monkeypatch.setenv("SRT_POOL", "1")
    b, p, st2 = gpu_render(setup, 16)
    assert bits_equal(a, b).all() and (o == p).all() and st["rays"] == st2["rays"]


@pytest.mark.parametrize("scene", ["rubik", "spheres", "global"])
def test_pipelined_launches_match_one_stream(rubik, monkeypatch, scene):
    """Pipelined sample launches (SRT_PIPELINE slots, each its own stream and launch buffers; launches
    overlapping each other or in series, SRT_PIPELINE_OVERLAP): renders enqueued back to back, in many small chunks (a small sample buffer) so that every slot is reused with
    its tile order from its previous launch, give the frame of the one-stream build bit for bit; and
    srt_kernel_time counts every launch."""
    if scene == "global":
        monkeypatch.setenv("SRT_FORCE_GLOBAL_SCENE", "1")
    setup = (R.make_setup(56, 40, show_model=False, max_depth=4) if scene == "spheres"
             else R.make_setup(56, 40, show_model=True, models=[rubik]))
    got = {}
    for pipe, overlap in (("1", "1"), ("3", "2"), ("2", "2"), ("3", "1")):  # 1: overlap only for nranks > 1
        monkeypatch.setenv("SRT_PIPELINE", pipe)
        monkeypatch.setenv("SRT_PIPELINE_OVERLAP", overlap)
        # 3 frames per chunk: SRT_SAMPLE_BUFFER_* is the context's whole budget, split over its own sample
        # buffer and one per pipeline slot
        nbuf = int(pipe) + 1 if int(pipe) > 1 else 1
        monkeypatch.setenv("SRT_SAMPLE_BUFFER_KB", str(56 * 40 * 16 * 3 * nbuf // 1024 + 1))
        r = R.Renderer(setup)
        try:
            r.compute.kernel_time()
            for _ in range(3):  # no finish between the renders
                r.render(16, write_output=True)
            r.finish()
            ms, launches = r.compute.kernel_time()
            assert launches == 3 * 6 and ms > 0.0  # 16 frames in chunks of 3: 6 launches per render
            assert r.compute.GetInt("launch.chunks") == 6
            assert r.compute.GetInt("launch.overlap") == (1 if pipe != "1" and overlap == "2" else 0)
            got[pipe + "/" + overlap] = (r.accum(), r.output())
        finally:
            r.close()
    for key in ("3/2", "2/2", "3/1"):
        assert bits_equal(got[key][0], got["1/1"][0]).all(), f"SRT_PIPELINE/OVERLAP={key}"
        assert (got[key][1] == got["1/1"][1]).all()
    acc, out, _ = oracle_render(setup, 16)
    assert bits_equal(got["3/2"][0], acc).all() and (got["3/2"][1] == out).all()
