"""Pin the CPU oracle and the arithmetic contract (CPU only).

Known answers come from the reference's own test scene (Rubik, the ray KAT of
include/compute/tests/BVH_intergration_tests.cpp:66-94 re-derived in SURVEY.md
8c) and from the glibc stream the reference's noise comes from.
"""
import math

import numpy as np
import pytest

from oracle import pyoracle as O
from oracle import scene_ref as REF


def test_sin_cos_accuracy():
    """The contract's fp32 sin/cos stay within 2 ulp of the true values."""
    rng = np.random.default_rng(2)
    xs = np.concatenate([rng.uniform(-4, 4, 4000), rng.uniform(-1e4, 1e4, 4000), rng.uniform(-1e6, 1e6, 2000),
                         np.array([0.0, -0.0, 1e-30, 3.14159265, 1.5707964, 1e5, -1e6], np.float64)])
    for x in xs.astype(np.float32):
        for got, want in ((O.sin(x), math.sin(float(x))), (O.cos(x), math.cos(float(x)))):
            ulp = float(np.spacing(np.float32(abs(want)))) if want != 0.0 else 1e-45
            assert abs(got - want) <= 2.0 * ulp, (x, got, want)


def test_sin_special_values():
    assert math.isnan(O.sin(float("nan"))) and math.isnan(O.sin(float("inf")))
    assert O.sin(2.0e9) == 0.0  # |x| >= 2^30: defined as 0


def test_pow_accuracy_and_glsl_domain():
    for x in np.concatenate([np.linspace(1e-6, 2.0, 997), np.array([1e-38, 1e-42, 1.0, 0.5])]).astype(np.float32):
        for y in (5.0, 1.0 / 2.4):
            want = float(x) ** float(np.float32(y))
            got = O.pow(float(x), float(np.float32(y)))
            assert abs(got - want) <= 1.5e-7 * abs(want) + 1e-44, (x, y, got, want)
    assert math.isnan(O.pow(-0.25, 5.0))      # exp2(y*log2(x)) with x < 0
    assert O.pow(0.0, 5.0) == 0.0
    assert math.isnan(O.pow(float("nan"), 5.0))


def _rn32_pow5(x):
    """x^5 rounded to nearest-even fp32, from the exact integer value (normal results only)."""
    m, e = math.frexp(float(x))          # x = m * 2^e, 0.5 <= m < 1
    mi = int(m * (1 << 24))              # 24-bit integer mantissa: x = mi * 2^(e - 24)
    p = mi ** 5
    shift = p.bit_length() - 24
    q, rem = p >> shift, p & ((1 << shift) - 1)
    half = 1 << (shift - 1)
    if rem > half or (rem == half and q & 1):
        q += 1
    return float(np.float32(math.ldexp(q, shift + 5 * (e - 24))))


def test_pow5_is_correctly_rounded():
    """pow(x, 5.0) of the Fresnel terms: x^5 rounded to nearest-even."""
    rng = np.random.default_rng(5)
    xs = np.concatenate([rng.uniform(0.001, 1.0, 4000), rng.uniform(1.0, 30.0, 1000),
                         np.array([1.8125, 0.90625, 0.453125, 29.0, 0.001, 1.0, 0.5])]).astype(np.float32)
    for x in xs:
        assert O.pow5(float(x)) == _rn32_pow5(x), x
    # 1.8125^5 = 29^5 / 2^20 lies exactly halfway between two floats: ties to even
    assert O.pow5(1.8125) == _rn32_pow5(1.8125) == float(np.float32(20511148 / 2**20))
    assert math.isnan(O.pow5(-0.25)) and math.isnan(O.pow5(float("nan")))
    assert O.pow5(0.0) == 0.0 and math.copysign(1.0, O.pow5(-0.0)) == 1.0
    assert O.pow5(float("inf")) == float("inf") and O.pow5(1e30) == float("inf")


def test_rand_float_is_fract_of_scaled_sin():
    for sx, sy in ((0.0, 0.0), (1.25, -3.5), (17.0, 9.0), (-8.7238, 5.9055)):
        # dot(seed, vec2(12.9898, 78.233)) under the contract: fma(sy, 78.233, sx * 12.9898)
        d = REF.fma_f32(np.float32(sy), np.float32(78.233), np.float32(np.float32(sx) * np.float32(12.9898)))
        m = np.float32(np.float32(O.sin(float(d))) * np.float32(43758.5453))
        want = np.float32(m - np.float32(math.floor(m)))
        assert O.rand_float(sx, sy) == float(want)


KAT_ODD = ((-10.0, 3.0, 6.0), (0.9838, -0.0118, 0.1787))   # BVH_intergration_tests.cpp:74
KAT_EVEN = ((0.0, 0.0, 0.0), (0.0, 1.0, 0.0))             # :76


def kat_rays(n=64):
    """The reference test's 64 rays (BVH_intergration_tests.cpp:69-77): odd rays KAT_ODD, even rays KAT_EVEN,
    intersection_distance 1e30 (Common::Ray, common/types.h:32)."""
    import srt_amd as S

    rays = np.zeros(n, S.RAY_DTYPE)
    for i in range(n):
        o, d = KAT_ODD if i % 2 else KAT_EVEN
        rays[i]["o"], rays[i]["d"] = o, np.array(d, np.float32)
    rays["t"] = 1e30
    return rays


def test_closest_hit_kat_on_rubik(rubik_scene):
    """BVH_intergration_tests.cpp:66-94 rays through the oracle: the odd ray's hit, distance and traversal
    counts, the even ray's hit (below)."""
    rays = kat_rays(2)[::-1].copy()          # [odd, even]
    orc = O.Oracle(rubik_scene)
    hits, t, n, st = orc.trace_closest(1, rays[:1])
    assert hits[0] == 365
    assert abs(t[0] - 1.0030496) < 2e-7
    assert st["nodes"] == 51 and st["tris"] == 91 and st["max_stack"] == 8
    hits, t, n, _ = orc.trace_closest(1, rays[1:])
    assert hits[0] == 331
    assert abs(t[0] - 5.9054995) < 2e-7


def test_reference_kat_odd_ray_hits_loader_triangle_17(rubik_scene):
    """The reference's own expected value pins the oracle: BVH_intergration_tests.cpp:94 expects every odd
    ray to hit triangle **17**.  The traversal returns the BVH-order index (ray_intersects.glsl:121), 365;
    BVH<Triangle> permuted the loader's triangles (bvh.h:66-72), and 365 is the loader's all_triangles[17]
    (model_loader.cpp:299-331): the expected value is stated in loader order, and the oracle's traversal hits
    exactly that triangle (1 in 1188 by chance).  The permutation comes from the C ABI
    (srt_scene_tri_order / srt_model_prim_order) and, independently, from oracle/scene_ref.py's restatement
    of bvh.h."""
    from conftest import OBJECTS

    rays = kat_rays(64)
    hits, _, _, _ = O.Oracle(rubik_scene).trace_closest(1, rays)
    odd = hits[1::2]
    assert (odd == 365).all()
    assert (rubik_scene.tri_input[odd] == 17).all()            # the reference's expected value, :94
    assert (rubik_model().prim_order() == rubik_scene.tri_input).all()
    packed, tris, _, _ = REF.load_obj(OBJECTS / "Rubik" / "Rubik.obj")
    _, prims, _, order = REF.build_bvh(packed, tris, with_order=True)
    assert order[365] == 17 and prims[365] == tris[17]
    assert (np.asarray(order, np.uint32) == rubik_scene.tri_input).all()


def test_reference_kat_even_ray_disagreement(rubik_scene):
    """BVH_intergration_tests.cpp:76,94 expects the even ray (o = 0, d = +Y) to miss.  It hits the top face of
    the bottom centre cubie (loader triangle 176) at t = 5.9054995 under every reading tried: recorded as an
    unexplained disagreement ("What is pinned").  The candidates, oracle only:
    - every arithmetic contract A-E (FMA in dot/cross or not, every a*b+c fused, sin in double);
    - the 1e-4 epsilon of intersection_utils_test.cpp:36 (the hit's t is 5.9, far above either epsilon, so
      the closest accepted hit cannot change);
    - the origin on the root box's bottom plane (min y = 0): nudged by +-1e-6, 1 denormal ulp, or below;
    - the ghost bvh_count = 2 of src/main.cpp:683 (its zero record never hits);
    - GLSL min/max NaN semantics: no node on this ray has an x or z bound of 0, so the slab test's
      0 * inf never occurs and no NaN enters it."""
    import srt_amd as S

    rays = kat_rays(2)[:1]
    for c in O.CONTRACTS:
        h, t, _, _ = O.Oracle(rubik_scene, contract=c).trace_closest(1, rays)
        assert h[0] == 331 and rubik_scene.tri_input[h[0]] == 176 and abs(t[0] - 5.9054995) < 2e-7, c
    assert t[0] > 1e-4
    mn, mx = np.stack(rubik_scene.nodes["min"]), np.stack(rubik_scene.nodes["max"])
    assert not ((mn[:, [0, 2]] == 0) | (mx[:, [0, 2]] == 0)).any()
    assert mn[0][1] == 0.0
    nudged = np.zeros(4, S.RAY_DTYPE)
    for i, oy in enumerate((1e-6, -1e-6, float(np.nextafter(np.float32(0), np.float32(1))), -1e-3)):
        nudged[i]["o"], nudged[i]["d"] = (0.0, oy, 0.0), (0.0, 1.0, 0.0)
    nudged["t"] = 1e30
    for bvh_count in (1, 2):
        h, t, _, _ = O.Oracle(rubik_scene).trace_closest(bvh_count, np.concatenate([rays, nudged]))
        assert (h != 0xFFFFFFFF).all(), bvh_count
        assert (rubik_scene.tri_input[h[:4]] == 176).all()     # from below the bottom plane it hits that face


def test_model_matrix_moves_scene_away(rubik_scene):
    """BVH_intergration_tests.cpp:97-113: after UpdateModelMatrix(mat4(1e-6) with [c][3] set) every ray misses."""
    import srt_amd as S

    sc = rubik_scene
    bvhs = sc.bvhs.copy()
    m = np.full((4, 4), np.float32(0.000001), np.float32)  # glm::mat4(0.000001f): diagonal only
    m[:] = 0.0
    for i in range(4):
        m[i, i] = 0.000001
    m[0, 3], m[1, 3], m[2, 3] = 10, 1000, 10  # new_mat[c][3]
    bvhs[0]["frame"] = m.reshape(16)
    moved = S.Scene(bvhs, sc.nodes, sc.mats, sc.tex_albedo, sc.tris, sc.verts)
    rays = np.zeros(64, S.RAY_DTYPE)
    for i in range(64):
        if i % 2:
            rays[i]["o"], rays[i]["d"] = (-10.0, 3.0, 6.0), np.array([0.9838, -0.0118, 0.1787], np.float32)
        else:
            rays[i]["o"], rays[i]["d"] = (0.0, 0.0, 0.0), (0.0, 1.0, 0.0)
        rays[i]["t"] = 1e30
    hits, _, _, _ = O.Oracle(moved).trace_closest(1, rays)
    assert (hits == 0xFFFFFFFF).all()


def test_golden_oracle_renders(rubik_scene):
    """Tiny oracle renders, pinned against committed fixtures: regression guard."""
    import json
    import hashlib
    from conftest import GOLDEN, oracle_render
    from srt_amd import render as R

    golden = json.loads((GOLDEN / "oracle_renders.json").read_text())
    for case in golden["cases"]:
        models = [rubik_model()] if case["scene"] == "rubik" else None
        setup = R.make_setup(case["width"], case["height"], show_model=case["scene"] == "rubik", models=models,
                             max_depth=case["max_depth"])
        acc, out, st = oracle_render(setup, case["spp"])
        assert hashlib.sha256(acc.tobytes()).hexdigest() == case["accum_sha256"], case
        assert hashlib.sha256(out.tobytes()).hexdigest() == case["out_sha256"], case
        assert st["rays"] == case["rays"]


def rubik_model():
    from conftest import OBJECTS
    import srt_amd as S

    return S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")


@pytest.fixture(scope="module")
def rubik_scene():
    import srt_amd as S

    return S.Scene.from_models([rubik_model()])
