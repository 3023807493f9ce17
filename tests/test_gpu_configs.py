"""GPU parity at BASELINE.json's configurations (C1, C2, C4, C5) and on the kernel instances the
small-scene tests do not reach.

Bar (as in test_gpu_parity.py): the HIP accumulation image bit-identical to the CPU oracle (NaN ==
NaN), the RGBA8 image identical.  Where a full-frame oracle render would take minutes, the oracle
renders rows spread across the frame at the config's full spp, and size-independent properties
cover the rest: determinism of two full renders, and the 8-rank row-band split (rendered rank by
rank on one GPU, reassembled by srt_assemble_bands) bit-identical to the 1-rank frame.

Configs (BASELINE.json "configs"):
  C1 sphere scene 256x256 @ 1 spp (maxDepth 5)              -- full frame vs the oracle
  C2 sphere scene 1024x1024 @ 64 spp, maxDepth 4            -- full render, oracle rows
  C3 Airplane OBJ 1920x1080 @ 256 spp                       -- blocked: the .obj is absent from the
                                                               reference checkout (.MISSING_LARGE_BLOBS);
                                                               its materials are pinned by test_airplane_*
  C4 Rubik 4096x4096 @ 1024 spp, maxDepth 8, 8 ranks        -- full render, oracle rows at 1024 spp,
                                                               8-way band split reassembled
  C5 synthetic 10 M triangles 4096x4096 (512 spp in the config) -- full frame at the bench's 16 spp,
                                                               oracle rows, determinism
  C5 at its configured 512 spp                               -- full frame, counting vs timed IL instance,
                                                               oracle rows at 512 spp
  C3 stand-in: torus-knot surface mesh 1920x1080 @ 256 spp      -- C3's regime (global-scene mode, real
                                                               surface mesh) at C3's size, oracle rows
  C3 stand-in with the Airplane's material set               -- the same surface carrying the Airplane's six
                                                               .mtl materials and PNG textures, sampled at
                                                               real uvs (the TEX instance), 1080p @ 256 spp
Every render goes through the counting instance and then the timed instance the benchmark measures at
that size, which must agree bit for bit.
"""
import numpy as np
import pytest

import srt_amd as S
from srt_amd import parallel as PAR
from srt_amd import render as R
from conftest import OBJECTS, bits_equal, oracle_render

pytestmark = pytest.mark.gpu


def gpu_render(setup, spp, *, timed=True, count=True, **kw):
    """The frame through the counting instance (with its CheckHit counts), then again through the timed
    instance bench.py measures at this size (sphere_kernel, the LDS kernel, global-scene mode's fused or IL
    instance at the scene's wave count), which must give the same frame bit for bit.  count=False renders
    the timed instance alone (stats empty)."""
    r = R.Renderer(setup, **kw)
    try:
        acc = out = None
        st = {}
        if count:
            r.render(spp, count=True)
            r.finish()
            acc, out, st = r.accum(), r.output(), r.compute.stats()
        if timed or not count:
            r.render(spp)
            r.finish()
            tacc, tout = r.accum(), r.output()
            if acc is not None:
                eq = bits_equal(tacc, acc)
                assert eq.all(), f"timed instance: {(~eq).sum()} accumulation values differ from the counting one"
                assert (tout == out).all()
            acc, out = tacc, tout
        return acc, out, st
    finally:
        r.close()


def timed_instance(setup) -> str:
    """The instance bench.py's timed launches take for this setup (srt_get_int's scene.* names)."""
    r = R.Renderer(setup)
    try:
        c = r.compute
        if not setup.show_model:
            return "sphere"
        return f"fused{c.GetInt('scene.global_waves')}" if c.GetInt("scene.fused") == 1 else "IL"
    finally:
        r.close()


def spread_rows(height, n):
    """n rows spread over the frame, first and last included."""
    return np.unique(np.linspace(0, height - 1, n).round().astype(np.int32))


def assert_rows(gacc, gout, acc, out, rows):
    eq = bits_equal(gacc[rows], acc[rows])
    assert eq.all(), f"{(~eq).sum()} accumulation values differ on the sampled rows"
    assert (gout[rows] == out[rows]).all()


def test_c1_spheres_256_1spp_full_frame():
    setup = R.make_setup(256, 256, show_model=False, max_depth=5)
    acc, out, st = oracle_render(setup, 1)
    gacc, gout, gst = gpu_render(setup, 1)
    assert bits_equal(gacc, acc).all()
    assert (gout == out).all()
    assert gst["rays"] == st["rays"] and gst["samples"] == 256 * 256 and gst["stack_overflow"] == 0


def test_c2_spheres_1024_64spp_depth4():
    setup = R.make_setup(1024, 1024, show_model=False, max_depth=4)
    assert timed_instance(setup) == "sphere"
    gacc, gout, gst = gpu_render(setup, 64)
    rows = spread_rows(1024, 24)
    acc, out, st = oracle_render(setup, 64, rows=rows)
    assert_rows(gacc, gout, acc, out, rows)
    assert gst["samples"] == 1024 * 1024 * 64 and gst["stack_overflow"] == 0
    assert np.isfinite(gacc[..., :3]).all() and (gacc[..., 3] == 1.0).all()


def _assemble(setup, parts, band, spp):
    """The root side of bench.py's step: srt_assemble_bands over the ranks' packed rows."""
    import torch

    W, H = setup.width, setup.height
    nranks = len(parts)
    rows_pad = PAR.rows_pad(H, band, nranks)
    gathered = torch.zeros((nranks, rows_pad, W, 4), dtype=torch.float32, device="cuda")
    for rank, loc in enumerate(parts):
        gathered[rank, :loc.shape[0]] = torch.from_numpy(loc).cuda()
    torch.cuda.synchronize()
    r = R.Renderer(setup)
    try:
        acc = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        out = torch.empty((H, W), dtype=torch.int32, device="cuda")
        r.compute.assemble_bands(gathered.data_ptr(), nranks, rows_pad, band, spp + 1, acc.data_ptr(),
                                 out.data_ptr())
        r.finish()
        torch.cuda.synchronize()
        return acc.cpu().numpy(), out.cpu().numpy().view(np.uint8).reshape(H, W, 4)
    finally:
        r.close()


def test_c4_rubik_4096_1024spp_depth8_rows_and_8_rank_split():
    W = H = 4096
    spp = 1024
    setup = R.make_setup(W, H, show_model=True, models=[R.rubik_model(OBJECTS)], max_depth=8)
    gacc, gout, gst = gpu_render(setup, spp)
    assert gst["samples"] == W * H * spp and gst["stack_overflow"] == 0
    rows = spread_rows(H, 16)
    acc, out, _ = oracle_render(setup, spp, rows=rows)
    assert_rows(gacc, gout, acc, out, rows)
    # the 8-GPU split of the config, rank by rank on one GPU (bench.py's 2-row bands)
    band, nranks = 2, 8
    parts = [gpu_render(setup, spp, count=False, rank=r, nranks=nranks, band_rows=band)[0] for r in range(nranks)]
    facc, fout = _assemble(setup, parts, band, spp)
    assert bits_equal(facc, gacc).all()
    assert (fout == gout).all()


@pytest.fixture(scope="module")
def c5_setup():
    model = R.synthetic_model(10_000_000)
    info = model.info()
    assert info["triangles"] == 10_000_000
    return R.make_setup(4096, 4096, show_model=True, models=[model])


def test_c5_synthetic_10M_rows_and_determinism(c5_setup):
    """C5 at its full frame size and scene, at the bench's 16 spp of its 512 (the rate, not the image, is the
    config's point): the counting and the timed IL instance (tile-major order, compiled in only for trees
    past 600 MB) bit-equal, oracle rows across the frame, and two full renders identical."""
    setup = c5_setup
    assert timed_instance(setup) == "IL"
    spp = 16
    a, o, st = gpu_render(setup, spp)
    assert st["samples"] == 4096 * 4096 * spp and st["stack_overflow"] == 0
    assert st["max_stack"] > 0
    rows = spread_rows(4096, 6)
    acc, out, _ = oracle_render(setup, spp, rows=rows)
    assert_rows(a, o, acc, out, rows)
    b, p, _ = gpu_render(setup, spp, count=False)
    assert bits_equal(a, b).all() and (o == p).all()


def test_c5_synthetic_10M_512spp_full_config(c5_setup):
    """C5 as BASELINE.json configures it: 4096x4096 @ 512 spp on the 10 M-triangle scene.  The counting
    instance and the timed IL instance agree bit for bit over the whole frame (both run every one of the
    512 frames, in 16-GiB sample-buffer chunks), and the oracle renders three rows at 512 spp."""
    setup = c5_setup
    spp = 512
    a, o, st = gpu_render(setup, spp)
    assert st["samples"] == 4096 * 4096 * spp and st["stack_overflow"] == 0 and st["bounce_cap"] == 0
    rows = spread_rows(4096, 3)
    acc, out, _ = oracle_render(setup, spp, rows=rows)
    assert_rows(a, o, acc, out, rows)
    assert np.isfinite(a[..., :3]).all()


AIRPLANE_MATERIALS = ("11803_Airplane_body", "11803_Airplane_wing_R", "11803_Airplane_wing_details_R",
                      "11803_Airplane_tail", "11803_Airplane_wing_details_L", "11803_Airplane_wing_L")


def test_c3_standin_airplane_materials_textured_1080p_256spp(tmp_path):
    """C3's material path at C3's size (it ran only at 48x40): the 262,144-triangle surface
    carries the Airplane's own six .mtl materials and 1024x1024 diffuse PNGs (tests/golden/objects, the
    reference's assets), one segment of the knot each, with real per-vertex uvs (the loader with
    has_texcoords set), so every hit samples its material's texture bilinearly at its interpolated uv
    (TriangleToSupportedMat, raytrace_utils.glsl:140-175).  Its faces are wound outward, as an exported
    model's are, so paths bounce off the surface and sample textures at their bounce hits too.  1920x1080 @ 256 spp through the timed texture
    instance of global-scene mode (fused, 5 waves per SIMD), bit-equal to the counting instance over the
    frame and to the oracle on rows spread across it."""
    import shutil

    src = OBJECTS / "11803_Airplane_v1_l1"
    for f in src.iterdir():
        shutil.copy(f, tmp_path / f.name)
    obj = R.write_textured_torus_knot_obj(tmp_path / "knot_airplane.obj", "11803_Airplane_v1_l1.mtl",
                                          AIRPLANE_MATERIALS)
    model = S.load_obj(obj, texcoords=True)
    assert model.info()["materials"] == 6 and model.info()["triangles"] == 262144
    setup = R.make_setup(1920, 1080, show_model=True, models=[model])
    sc = setup.scene
    assert sc.sample_textures and (sc.mats["use_texture"] == 1).all() and len(sc.textures) == 6
    assert float(sc.verts["uv"].max()) > 1.0  # uvs past 1: GL_REPEAT wrapping is exercised
    assert timed_instance(setup) == "fused5"
    spp = 256
    a, o, st = gpu_render(setup, spp)
    assert st["samples"] == 1920 * 1080 * spp and st["stack_overflow"] == 0
    assert st["mat_reads"] > 0
    # bounce rays: each shaded hit (one material read) traces a shadow ray and, off an outward face, mostly a
    # bounce ray as well (inward faces end the path after the shadow ray: about one secondary ray per hit)
    assert st["rays"] - st["samples"] > 1.3 * st["mat_reads"]
    rows = spread_rows(1080, 12)
    acc, out, _ = oracle_render(setup, spp, rows=rows)
    assert_rows(a, o, acc, out, rows)
    # the textures matter: the constant-albedo (uv = (0,0)) load of the same OBJ renders a different frame
    const = R.make_setup(1920, 1080, show_model=True, models=[S.load_obj(obj)])
    assert not const.scene.sample_textures
    ca, _, _ = oracle_render(const, 2, rows=rows)
    ta, _, _ = oracle_render(setup, 2, rows=rows)
    assert not bits_equal(ca[rows], ta[rows]).all()


def test_c3_standin_surface_mesh_1080p_256spp():
    """C3's regime (the Airplane OBJ is absent: .MISSING_LARGE_BLOBS): a real surface mesh in global-scene
    mode at C3's frame and spp, 1920x1080 @ 256 spp -- the bench's surface-mesh scene (torus-knot tube,
    262,144 triangles wound outward as an exported model is, framed at SURFACE_KNOT_SCALE; model camera and
    lights) through the timed fused instance at 5 waves per SIMD, bit-equal to the counting instance over the
    whole frame and to the oracle on rows spread across it.  Paths bounce off it (the inward
    knot of rounds 2-5 rejected every bounce at dot(N, V) <= 0, brdf.glsl:242): bounce rays are at least 20%
    of the counted rays (srt_ray_kinds), and the oracle's rows see the same ray mix."""
    setup = R.make_setup(1920, 1080, show_model=True, models=[R.torus_knot_model()])
    assert timed_instance(setup) == "fused5"
    spp = 256
    a, o, st = gpu_render(setup, spp)
    assert st["samples"] == 1920 * 1080 * spp and st["stack_overflow"] == 0
    bounce = st["rays"] - st["samples"] - st["shadow_rays"]
    assert bounce >= 0.20 * st["rays"], (bounce, st)
    rows = spread_rows(1080, 12)
    acc, out, ost = oracle_render(setup, spp, rows=rows)
    assert_rows(a, o, acc, out, rows)
    assert ost["rays"] - ost["samples"] - ost["shadow_rays"] >= 0.15 * ost["rays"]
    assert st["tris"] > st["samples"]  # (the mesh covers much of the frame: more triangle tests than samples)


def test_first_hit_only_knot_never_bounces():
    """The inward-wound knot the surface-mesh leg used in rounds 2-5 (render.first_hit_only_knot_model): every
    bounce is rejected (dot(N, V) <= 0, brdf.glsl:242), so its rays are camera and shadow rays only; the outward
    knot of the same grid bounces.  192x108 @ 4 spp, counting instance, against the oracle's counts."""
    for model, bounces in ((R.first_hit_only_knot_model(), False), (R.torus_knot_model(scale=1.0), True)):
        setup = R.make_setup(192, 108, show_model=True, models=[model])
        _, _, st = gpu_render(setup, 4, timed=False)
        _, _, ost = oracle_render(setup, 4)
        assert (st["rays"], st["shadow_rays"]) == (ost["rays"], ost["shadow_rays"])
        b = st["rays"] - st["samples"] - st["shadow_rays"]
        assert (b > 0.1 * st["rays"]) if bounces else (b < 1e-3 * st["rays"]), (b, st)


def _coincident_star(n=300, seed=5):
    """n triangles whose centroids are exactly (0, 6, 0): dyadic coordinates, so (p0 + p1 + p2) / 3
    is exact and the midpoint split can never separate them -- one leaf of n >= 256 triangles
    (bvh.h:129-130: a side is empty), which sends the scene to the unpacked 3-dword stack path."""
    rng = np.random.default_rng(seed)
    c = np.array([0.0, 6.0, 0.0], np.float32)
    a = rng.integers(-24, 25, size=(n, 3)).astype(np.float32) / np.float32(8.0)
    b = rng.integers(-24, 25, size=(n, 3)).astype(np.float32) / np.float32(8.0)
    tri = np.stack([c + a, c + b, c - a - b], axis=1)
    floor = np.array([[-30, 0, -30], [30, 0, -30], [30, 0, 30], [-30, 0, -30], [30, 0, 30], [-30, 0, 30]],
                     np.float32).reshape(2, 3, 3)
    return np.concatenate([floor, tri]).reshape(-1, 9)


def test_unpacked_stack_path_big_leaf():
    """A leaf of >= 256 triangles: global-scene mode with 3-dword (unpacked) stack entries."""
    model = S.model_from_triangles(_coincident_star(), kd=(0.7, 0.6, 0.5), ks=(0.2, 0.2, 0.2), ns=20.0)
    setup = R.make_setup(48, 40, show_model=True, models=[model])
    assert int(setup.scene.nodes["count"].max()) >= 256
    setup.camera.position = np.asarray((0.0, 7.0, 14.0), np.float32)
    acc, out, st = oracle_render(setup, 3)
    gacc, gout, gst = gpu_render(setup, 3)
    assert bits_equal(gacc, acc).all()
    assert (gout == out).all()
    # (node / triangle counts differ by design: shadow rays stop at their first accepted triangle on the
    # GPU, while the oracle runs CheckLightOccluded's full closest-hit query; the result is the same)
    assert gst["rays"] == st["rays"] and gst["stack_overflow"] == 0


def test_unpacked_stack_path_closest_hit():
    from oracle import pyoracle as O

    model = S.model_from_triangles(_coincident_star(), kd=(0.7, 0.6, 0.5), ks=(0.2, 0.2, 0.2), ns=20.0)
    scene = S.Scene.from_models([model])
    rng = np.random.default_rng(3)
    rays = np.zeros(4000, S.RAY_DTYPE)
    rays["o"] = rng.uniform([-8, 1, -8], [8, 12, 8], size=(4000, 3)).astype(np.float32)
    tgt = np.array([0.0, 6.0, 0.0], np.float32) + rng.normal(scale=1.5, size=(4000, 3)).astype(np.float32)
    rays["d"] = (tgt - rays["o"]).astype(np.float32)
    rays["t"] = np.float32(1e30)
    hits_o, t_o, _, _ = O.Oracle(scene).trace_closest(1, rays)
    c = S.Compute().Init()
    try:
        c.bind_scene(scene)
        c.SetUInt("bvh_count", 1)
        hits, t = c.trace_closest(rays)
    finally:
        c.close()
    assert (hits == hits_o).all() and bits_equal(t, t_o).all()
    assert (hits >= 2).sum() > 1000  # most rays hit the coincident leaf, not the floor


def _deep_chain(n=200):
    """Triangles at x = 1.5^k: the midpoint split peels one or two off per level, so the tree is about
    n / 1.5 levels deep -- beyond the LDS stacks of both the closest-hit kernel (HBM stacks) and the
    sample kernel (global-scene mode with its LDS ring spilling to HBM)."""
    tri = []
    for k in range(n):
        x, s = np.float32(1.5) ** k, np.float32(0.3) * np.float32(1.5) ** k
        tri.append([[x - s, -s, 0.0], [x + s, -s, 0.0], [x, s, 0.0]])
    return np.asarray(tri, np.float32).reshape(-1, 9)


def test_deep_tree_closest_hit_and_render():
    from oracle import pyoracle as O

    model = S.model_from_triangles(_deep_chain(), kd=(0.6, 0.6, 0.6), ks=(0.1, 0.1, 0.1), ns=8.0)
    depth = model.info()["max_depth"]
    assert depth > 90
    scene = S.Scene.from_models([model])
    n = 200
    rays = np.zeros(2 * n, S.RAY_DTYPE)
    k = np.arange(n)
    x = np.float32(1.5) ** k.astype(np.float32)
    rays["o"][:n, 0] = x
    rays["o"][:n, 2] = np.float32(10.0) * x
    rays["d"][:n] = (0.0, 0.0, -1.0)
    rays["o"][n:] = (-2.0, 0.01, 0.0)
    rays["d"][n:, 0] = 1.0
    rays["d"][n:, 1] = np.linspace(-0.2, 0.2, n, dtype=np.float32)
    rays["t"] = np.float32(1e30)
    hits_o, t_o, _, _ = O.Oracle(scene).trace_closest(1, rays)
    c = S.Compute().Init()
    try:
        c.bind_scene(scene)
        c.SetUInt("bvh_count", 1)
        hits, t = c.trace_closest(rays)
    finally:
        c.close()
    assert (hits == hits_o).all() and bits_equal(t, t_o).all()
    assert (hits[:60] != 0xFFFFFFFF).all()  # (far out, M-T's absolute 1e-4 parallel test rejects)
    setup = R.make_setup(40, 32, show_model=True, models=[model])
    setup.camera.position = np.asarray((3.0, 0.5, 12.0), np.float32)
    acc, out, st = oracle_render(setup, 2)
    gacc, gout, gst = gpu_render(setup, 2)
    assert bits_equal(gacc, acc).all() and (gout == out).all()
    assert gst["rays"] == st["rays"] and gst["stack_overflow"] == 0


def test_deep_tree_hbm_stacks_past_2g_entries():
    """The closest-hit kernel's HBM stacks (trees too deep for LDS stacks) with more rays than a flat
    lane-interleaved layout could index in 32 bits: 9 M rays x 3 dwords x ~100 entries is past 2^31
    (ADVICE r02).  The 400 distinct rays of test_deep_tree_closest_hit_and_render are repeated; every
    copy must return the oracle's hit and distance."""
    from oracle import pyoracle as O

    model = S.model_from_triangles(_deep_chain(), kd=(0.6, 0.6, 0.6), ks=(0.1, 0.1, 0.1), ns=8.0)
    scene = S.Scene.from_models([model])
    depth = model.info()["max_depth"]
    n = 200
    base = np.zeros(2 * n, S.RAY_DTYPE)
    x = np.float32(1.5) ** np.arange(n).astype(np.float32)
    base["o"][:n, 0] = x
    base["o"][:n, 2] = np.float32(10.0) * x
    base["d"][:n] = (0.0, 0.0, -1.0)
    base["o"][n:] = (-2.0, 0.01, 0.0)
    base["d"][n:, 0] = 1.0
    base["d"][n:, 1] = np.linspace(-0.2, 0.2, n, dtype=np.float32)
    base["t"] = np.float32(1e30)
    hits_o, t_o, _, _ = O.Oracle(scene).trace_closest(1, base)
    reps = 22500  # 9,000,000 rays
    assert reps * len(base) * 3 * (depth + 1) > 2 ** 31
    rays = np.tile(base, reps)
    c = S.Compute().Init()
    try:
        c.bind_scene(scene)
        c.SetUInt("bvh_count", 1)
        hits, t = c.trace_closest(rays)
    finally:
        c.close()
    assert (hits.reshape(reps, -1) == hits_o).all()
    assert bits_equal(t.reshape(reps, -1), np.broadcast_to(t_o, (reps, len(base)))).all()
