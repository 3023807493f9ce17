"""Scene producers (host C++, libsrt_amd.so) vs the reference's known answers and vs an independent
Python restatement (oracle/scene_ref.py) -- bit for bit.  CPU only: no GPU call is made."""
import math
import pathlib
import subprocess

import numpy as np
import pytest

import srt_amd as S
from oracle import scene_ref as R
from conftest import OBJECTS

RUBIK = OBJECTS / "Rubik" / "Rubik.obj"


def test_rubik_ingest_known_answers():
    """SURVEY.md 8c item 1 (re-execution of the reference loader + builder on Rubik.obj)."""
    info = S.load_obj(RUBIK).info()
    assert info["triangles"] == 1188
    assert info["vertices"] == 3564
    assert info["nodes"] == 427
    assert info["leaves"] == 214
    assert info["max_depth"] == 9
    assert info["faces_dropped"] == 0
    np.testing.assert_array_equal(info["root_min"], np.array([-9.0132, 0.0, -9.1173], np.float32))
    np.testing.assert_array_equal(info["root_max"], np.array([9.1608, 18.3665, 9.1173], np.float32))


def _scene_from_ref(models):
    bvhs, nodes, mats, tris, verts = R.flatten(models)
    return bvhs, nodes, mats, tris, verts


def _compare_scene(sc: S.Scene, ref):
    bvhs, nodes, mats, tris, verts = ref
    assert len(sc.bvhs) == len(bvhs) and len(sc.nodes) == len(nodes) and len(sc.tris) == len(tris)
    assert len(sc.verts) == len(verts) and len(sc.mats) == len(mats)
    for i, (first, count) in enumerate(bvhs):
        assert sc.bvhs[i]["first_index"] == first and sc.bvhs[i]["count"] == count
        np.testing.assert_array_equal(sc.bvhs[i]["frame"], np.eye(4, dtype=np.float32).reshape(16))
    ref_nodes = np.zeros(len(nodes), S.NODE_DTYPE)
    for i, (mn, first, mx, count) in enumerate(nodes):
        ref_nodes[i] = (np.array(mn, np.float32), first, np.array(mx, np.float32), count)
    assert sc.nodes.tobytes() == ref_nodes.tobytes()
    ref_tris = np.array([(t[:3], t[3]) for t in tris], S.TRI_DTYPE)
    assert sc.tris.tobytes() == ref_tris.tobytes()
    np.testing.assert_array_equal(sc.verts["pos"].view(np.uint32), np.array(verts, np.float32).view(np.uint32))
    assert (sc.verts["uv"] == 0).all()  # has_texcoords is never set (asset_utils/types.h:105)
    for i, (kd, ns, ks, use_tex) in enumerate(mats):
        assert sc.mats[i]["diffuse"].tobytes() == np.array(kd, np.float32).tobytes()
        assert sc.mats[i]["Ks"].tobytes() == np.array(ks, np.float32).tobytes()
        assert np.float32(sc.mats[i]["Ns"]) == ns and sc.mats[i]["use_texture"] == use_tex


def _ref_model(path):
    packed, tris, mats, dropped = R.load_obj(path)
    nodes, prims, depth = R.build_bvh(packed, tris)
    return (packed, nodes, prims, mats), depth, dropped


def test_rubik_arrays_match_independent_restatement():
    ref_model, depth, dropped = _ref_model(RUBIK)
    assert depth == 9 and dropped == 0
    _compare_scene(S.Scene.from_models([S.load_obj(RUBIK)]), _scene_from_ref([ref_model]))


def test_two_model_rebasing():
    """Index rebasing across models (gpu_loader.cpp:107-130)."""
    m1, _, _ = _ref_model(RUBIK)
    m2, _, _ = _ref_model(RUBIK)
    _compare_scene(S.Scene.from_models([S.load_obj(RUBIK), S.load_obj(RUBIK)]), _scene_from_ref([m1, m2]))


def test_primitive_permutation_across_models():
    """srt_model_prim_order / srt_scene_tri_order: the BVH's permutation (bvh.h:66-72) of each model, offset by
    the model's triangles before it in the flattened scene.  Checked against oracle/scene_ref.py's restatement
    of the builder, and against the loader's per-corner vertex duplication (model_loader.cpp:302-331: loader
    triangle k owns vertices 3k..3k+2, so a BVH-order triangle's first vertex is 3 x its input index), for
    two OBJ models and a raw-triangle model (the parallel builder's size, serial and on 8 threads)."""
    from srt_amd import render as RD

    rub = S.load_obj(RUBIK)
    soup = S.model_from_triangles(RD.synthetic_triangles(70_000, seed=5))
    sc = S.Scene.from_models([rub, soup, rub])
    n_r = rub.info()["triangles"]
    n_s = soup.info()["triangles"]
    order_r, order_s = rub.prim_order(), soup.prim_order()
    assert sorted(order_r.tolist()) == list(range(n_r)) and sorted(order_s.tolist()) == list(range(n_s))
    want = np.concatenate([order_r, order_s + n_r, order_r + n_r + n_s]).astype(np.uint32)
    assert (sc.tri_input == want).all()
    assert (sc.tris["v"][:, 0] == 3 * sc.tri_input).all()  # every model duplicates vertices per corner
    packed, tris, _, _ = R.load_obj(RUBIK)
    _, _, _, idx = R.build_bvh(packed, tris, with_order=True)
    assert (np.asarray(idx, np.uint32) == order_r).all()


def test_null_model_raises():
    with pytest.raises(Exception):
        S.Scene.from_models([None])


OBJ_EDGE = """# edge cases of ParseOBJ (model_loader.cpp:35-177)
mtllib edge.mtl\r
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0.5 0.5 1
vt 0 0
vn 0 0 1
f 1 2 3
usemtl red
f 1/1/1 2/1/1 3/1/1 4/1/1
f 1 2 3 4 5
   f 1//1 3//1 5//1   \t
usemtl missing
f 2 3 5
usemtl blue
f 3 4 5
"""
MTL_EDGE = """newmtl red
Kd 1 0 0
Ks 0.5 0.5 0.5
Ns 20
newmtl blue
Kd 0 0 1
newmtl red
Kd 0 1 0
"""


def test_obj_parser_edge_cases(tmp_path):
    (tmp_path / "edge.obj").write_text(OBJ_EDGE)
    (tmp_path / "edge.mtl").write_text(MTL_EDGE)
    m = S.load_obj(tmp_path / "edge.obj")
    info = m.info()
    # 1 face before the first usemtl joins 'red'; the quad is fanned to 2; the 5-gon is dropped;
    # 1 face under 'missing' (index 0), 1 under 'blue'
    assert info["triangles"] == 6 and info["faces_dropped"] == 1
    ref_model, _, dropped = _ref_model(tmp_path / "edge.obj")
    assert dropped == 1
    sc = S.Scene.from_models([m])
    _compare_scene(sc, _scene_from_ref([ref_model]))
    # the duplicate 'newmtl red' left the parser on 'blue', whose Kd became (0,1,0)
    assert sc.mats[1]["diffuse"].tolist() == [0.0, 1.0, 0.0]


def test_synthetic_mesh_bvh_matches():
    from srt_amd.render import synthetic_triangles

    xyz9 = synthetic_triangles(600, seed=7)
    m = S.model_from_triangles(xyz9)
    packed = [tuple(np.float32(v) for v in xyz9[t, 3 * c:3 * c + 3]) for t in range(600) for c in range(3)]
    tris = [(3 * t, 3 * t + 1, 3 * t + 2, 0) for t in range(600)]
    nodes, prims, depth = R.build_bvh(packed, tris)
    mats = [{"Kd": (np.float32(0.8),) * 3, "Ks": (np.float32(0),) * 3, "Ns": np.float32(10), "tex": None}]
    _compare_scene(S.Scene.from_models([m]), R.flatten([(packed, nodes, prims, mats)]))
    assert m.info()["max_depth"] == depth


def test_glibc_rand_stream():
    want = [1804289383, 846930886, 1681692777, 1714636915, 1957747793]  # glibc rand(), seed 1
    assert S.glibc_rand(5).tolist() == want
    g = R.GlibcRand()
    assert [g() for _ in range(2000)] == S.glibc_rand(2000).tolist()
    assert float(np.float32(want[0]) / np.float32(2147483648.0)) == pytest.approx(0.840187728, abs=1e-9)


def test_glibc_rand_matches_libc():
    import ctypes
    import ctypes.util

    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.srand(1)
    assert [libc.rand() for _ in range(1000)] == S.glibc_rand(1000).tolist()


@pytest.mark.parametrize("gcc_order", [True, False])
def test_noise_matches_restatement(gcc_order):
    noise, noise_u = S.generate_noise(13, 11, gcc_order=gcc_order)
    rn, ru = R.generate_noise(13 * 11, gcc_order=gcc_order)
    assert noise.tobytes() == rn.tobytes() and noise_u.tobytes() == ru.tobytes()
    norms = np.linalg.norm(noise.astype(np.float64), axis=1)
    assert np.all(np.abs(norms - 1) < 1e-6) and np.all((noise_u >= 0) & (noise_u <= 1))


def test_camera_basis():
    cam = S.Camera(show_model=True)
    assert cam.position.tolist() == [0.0, 9.0, 40.0]
    f, u, r = R.camera_basis(-90.0, 0.0)
    assert cam.front.tobytes() == np.array(f, np.float32).tobytes()
    assert cam.up.tobytes() == np.array(u, np.float32).tobytes()
    assert cam.right.tobytes() == np.array(r, np.float32).tobytes()
    assert S.Camera(show_model=False).position.tolist() == [0.0, 1.0, 4.0]
    cam.Rotate(30.0, -20.0)
    f, u, r = R.camera_basis(-60.0, -20.0)
    assert cam.front.tobytes() == np.array(f, np.float32).tobytes()


def test_camera_height_rounding():
    """GetCamera's int(width / aspect) (raytrace_compute.glsl:50): 1080 survives."""
    for w, h in ((1920, 1080), (1000, 800), (4096, 4096), (256, 256), (1024, 1024)):
        aspect = np.float32(w) / np.float32(h)
        assert int(np.float32(w) / aspect) == h


def _write_png(path, w, h, pixels, ctype=2):
    import struct
    import zlib

    ch = {0: 1, 2: 3, 6: 4}[ctype]
    raw = b"".join(b"\x00" + bytes(pixels[y * w * ch:(y + 1) * w * ch]) for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    path.write_bytes(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0))
                     + chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))


def test_texture_corner_albedo(tmp_path):
    """texture(sampler2D, uv=(0,0)) with GL_REPEAT + GL_LINEAR = mean of the four corner texels."""
    w, h = 5, 4
    px = [0] * (w * h * 3)

    def put(x, y, rgb):
        px[(y * w + x) * 3:(y * w + x) * 3 + 3] = rgb

    put(0, 0, (255, 0, 0)); put(w - 1, 0, (0, 255, 0)); put(0, h - 1, (0, 0, 255)); put(w - 1, h - 1, (255, 255, 255))
    _write_png(tmp_path / "t.png", w, h, px)
    (tmp_path / "m.mtl").write_text("newmtl tex\nKd 1 1 1\nNs 30\nmap_Kd t.png\n")
    (tmp_path / "m.obj").write_text("mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl tex\nf 1 2 3\n")
    sc = S.Scene.from_models([S.load_obj(tmp_path / "m.obj")])
    assert sc.mats[0]["use_texture"] == 1
    np.testing.assert_allclose(sc.tex_albedo[0], [0.5, 0.5, 0.5], atol=1e-7)


def _np_sample(tex, s, t):
    """The sampling contract restated in numpy float32: level 0, GL_LINEAR, GL_REPEAT."""
    f = np.float32
    h, w, ch = tex.shape
    s, t = f(s), f(t)
    s = s if np.isfinite(s) else f(0)
    t = t if np.isfinite(t) else f(0)
    s = f(s - np.floor(s))
    t = f(t - np.floor(t))
    x, y = f(s * f(w) - f(0.5)), f(t * f(h) - f(0.5))
    fx, fy = np.floor(x), np.floor(y)
    a, b = f(x - fx), f(y - fy)
    i0, j0 = int(fx), int(fy)
    i1, j1 = (i0 + 1) % w, (j0 + 1) % h
    i0, j0 = i0 % w, j0 % h
    wt = [f(f(1) - a) * f(f(1) - b), a * f(f(1) - b), f(f(1) - a) * b, a * b]

    def texel(i, j, k):
        if k >= ch or (ch == 2 and k == 2):
            return f(0)
        return f(f(tex[j, i, k]) / f(255))

    out = np.zeros(3, np.float32)
    for k in range(3):
        acc = f(wt[0] * texel(i0, j0, k))
        acc = f(acc + f(wt[1] * texel(i1, j0, k)))
        acc = f(acc + f(wt[2] * texel(i0, j1, k)))
        out[k] = f(acc + f(wt[3] * texel(i1, j1, k)))
    return out


@pytest.mark.parametrize("w,h,ch", [(1, 1, 3), (5, 4, 1), (7, 3, 2), (8, 8, 3), (3, 9, 4)])
def test_texture_sampler_contract(w, h, ch):
    """srt_texture_sample (csrc/scene.cpp TextureSample) against a numpy restatement of the contract, bit for bit,
    over ordinary, wrapped, boundary and non-finite coordinates."""
    rng = np.random.default_rng(w * 100 + h * 10 + ch)
    tex = rng.integers(0, 256, (h, w, ch), dtype=np.uint8)
    pts = list(rng.uniform(-3, 3, (40, 2)).astype(np.float32))
    pts += [(0, 0), (1, 1), (-0.0, 0.5), (0.999999, 1e-9), (-1e-9, -1e-9), (1e20, -1e20), (np.nan, 0.25),
            (np.inf, -np.inf), ((0.5 + 2) / w, (0.5 + 1) / h)]
    for s, t in pts:
        got = S.texture_sample(tex, s, t)
        want = _np_sample(tex, s, t)
        assert (got.view(np.uint32) == want.view(np.uint32)).all(), (s, t, got, want)
    # a texel centre returns that texel exactly
    i, j = w // 2, h // 2
    c = S.texture_sample(tex, np.float32((i + 0.5) / w), np.float32((j + 0.5) / h))
    exp = [tex[j, i, k] / np.float32(255) if k < ch and not (ch == 2 and k == 2) else 0 for k in range(3)]
    np.testing.assert_array_equal(c, np.float32(exp))


def test_unorm8_read_is_the_correctly_rounded_quotient():
    """The kernel keeps texels as RGBA8 and reads a channel c as q = c * RN(1/255) corrected once by
    fma(fma(-255, q, c), RN(1/255), q) (shading.hpp unorm8): for every byte that is c / 255.0f, the value
    the contract (and the host sampler above) uses.  fmaf from libm: one rounding, like the device's."""
    import ctypes
    fmaf = ctypes.CDLL("libm.so.6").fmaf
    fmaf.argtypes = [ctypes.c_float] * 3
    fmaf.restype = ctypes.c_float
    f = np.float32
    r = f(1) / f(255)
    assert r == f(0.003921568859368563)
    for c in range(256):
        q = f(f(c) * r)
        got = f(fmaf(fmaf(-255.0, q, float(c)), r, q))
        assert got.view(np.uint32) == (f(c) / f(255)).view(np.uint32), c


OBJ_UV = """mtllib m.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
vt 0.1 0.2
vt 0.9 0.2
vt 0.9 0.8
vt 0.1 0.8
usemtl tex
f 1/1 2/2 3/3 4/4
f 1//1 2//1 3//1
f 1/4/1 3/2/1 4/1/1
"""


def test_loader_texcoords(tmp_path):
    """vt indices per corner (model_loader.cpp:65-71,82-143): the quad's second triangle takes vt 1, 3, 4; a face
    without vt keeps (0,0); the default loader (has_texcoords never set, types.h:105) keeps every uv at (0,0)."""
    _write_png(tmp_path / "t.png", 2, 2, [10, 20, 30] * 4)
    (tmp_path / "m.mtl").write_text("newmtl tex\nKd 1 1 1\nNs 30\nmap_Kd t.png\n")
    (tmp_path / "m.obj").write_text(OBJ_UV)
    plain = S.Scene.from_models([S.load_obj(tmp_path / "m.obj")])
    assert (plain.verts["uv"] == 0).all() and not plain.sample_textures
    sc = S.Scene.from_models([S.load_obj(tmp_path / "m.obj", texcoords=True)])
    assert sc.sample_textures and len(sc.textures) == 1 and sc.textures[0].shape == (2, 2, 3)
    assert sc.mats[0]["use_texture"] == 1 and tuple(sc.mats[0]["handle"]) == (0, 0)
    vt = [(0.1, 0.2), (0.9, 0.2), (0.9, 0.8), (0.1, 0.8)]
    P = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0)]
    z = (0, 0)
    want = [(P[0], P[1], P[2], vt[0], vt[1], vt[2]), (P[0], P[2], P[3], vt[0], vt[2], vt[3]),
            (P[0], P[1], P[2], z, z, z), (P[0], P[2], P[3], vt[3], vt[1], vt[0])]
    got = []
    for tri in sc.tris:  # BVH order: compare as a multiset
        c = list(tri["v"])
        got.append(tuple(tuple(float(x) for x in sc.verts["pos"][i]) for i in c)
                   + tuple(tuple(float(x) for x in sc.verts["uv"][i]) for i in c))
    f = lambda e: tuple(tuple(float(np.float32(x)) for x in v) for v in e)  # noqa: E731
    assert sorted(got) == sorted(f(e) for e in want)


def test_missing_obj_raises(tmp_path):
    with pytest.raises(S.SrtError):
        S.load_obj(tmp_path / "nope.obj")


@pytest.mark.parametrize("n_tris", [70_000, 300_000])
def test_parallel_bvh_builder_is_bit_identical(monkeypatch, n_tris):
    """the parallel builder (csrc/scene.cpp BvhBuilder::BuildParallel) reproduces the
    reference's serial build (bvh.h:98-148) node for node and in primitive order."""
    import hashlib

    from srt_amd import render as R

    tri = R.synthetic_triangles(n_tris, seed=11)
    digests = []
    for threads in ("1", "8"):
        monkeypatch.setenv("SRT_BVH_THREADS", threads)
        m = S.model_from_triangles(tri)
        sc = S.Scene.from_models([m])
        digests.append((hashlib.sha256(sc.nodes.tobytes()).hexdigest(), hashlib.sha256(sc.tris.tobytes()).hexdigest(),
                        {k: v for k, v in m.info().items() if isinstance(v, int)}))
    assert digests[0] == digests[1]


FLOAT_EDGES = ["1 2 3", "1.0abc 2 3", "inf 1 2", "nan 1 2", "0x1p3 1 2", "1e40 1 2", "-1e40 1 2", "1e-40 2 3",
               "1e-50 2 3", "1e 2 3", "1.5e+ 2 3", ". 1 2", "- 1 2", "+.5 -.5e1 5.", "1 2", "1 2 3 4",
               "   7   8 9", "1,5 2 3", "00012.50e-01 2 3", "1e+ 2 3", "3.4028236e38 1 1", "3.4028235e38 1 1",
               "1.17549435e-38x 1 1", "1..2 3 4", "1e2e3 1 1", "-0 -0.0 +0", "0.1 0.2 0.3",
               "16777217 33554433.0 1.00000005960464477539062500000000001", "1.4e-45 7e-46 7.1e-46",
               "E5 1 1", "\t1\t2\t3", "123456789012345678901234567890 1 1", "-.e1 1 1", "1e-0 +1E+1 2e00"]


def test_istream_float_restatement_matches_libstdcxx():
    """oracle/scene_ref.py istream_floats vs `ls >> a >> b >> c` compiled here (tests/cpp/istream_probe.cpp):
    trailing garbage, inf/nan/hex words, overflow (+-FLT_MAX + failbit), underflow, halfway cases."""
    from test_boundary import _build

    exe = _build("istream_probe")
    res = subprocess.run([str(exe)], input="\n".join(FLOAT_EDGES) + "\n", capture_output=True, text=True, timeout=60)
    assert res.returncode == 0
    marker = np.float32(-12345.0)
    for line, got in zip(FLOAT_EDGES, res.stdout.split("\n")):
        ok, vals = R.istream_floats(line, 3)
        bits = [int(np.array(marker if v is None else v, np.float32).view(np.uint32)) for v in vals]
        assert got == f"{int(ok)} " + " ".join(f"{b:08x}" for b in bits), line


def test_obj_float_edge_lines(tmp_path):
    """Vertices and material lines whose numbers istream reads differently from a whole-token strtof: the
    C++ loader and the restatement agree vertex for vertex and material for material."""
    verts = ["v 0 0 0", "v 1 0 0", "v 1 1 0", "v 0 1 0", "v 1.0abc 2 3", "v inf 1 2", "v 1e40 0 0", "v 1..5 2 3",
             "v 1e-40 0.5 1e2e3", "v 2 2 2 junk", "v 0.3 0.7 1e-45"]
    obj = "mtllib e.mtl\nusemtl a\n" + "\n".join(verts) + "\nf 1 2 3\nf 1 3 4\nf 2 3 4\nf 4 5 6\nusemtl b\nf 1 2 4\n"
    mtl = ("newmtl a\nKd 0.5abc 0.25 1\nKs 1e40 2 3\nNs 7e\nnewmtl b\nKd 0x10 1 1\nKs .5 .25\nNs -1e40\n")
    (tmp_path / "e.obj").write_text(obj)
    (tmp_path / "e.mtl").write_text(mtl)
    m = S.load_obj(tmp_path / "e.obj")
    ref_model, _, _ = _ref_model(tmp_path / "e.obj")
    sc = S.Scene.from_models([m])
    _compare_scene(sc, _scene_from_ref([ref_model]))
    fmax = np.finfo(np.float32).max
    assert sc.mats[0]["diffuse"].tolist() == [0.5, 0.0, 0.0] and sc.mats[0]["Ks"][0] == fmax
    assert sc.mats[1]["diffuse"].tolist() == [0.0, 0.0, 0.0] and sc.mats[1]["Ns"] == -fmax
