"""the Airplane's materials, pinned by the reference's own assets.

The Airplane OBJ itself is absent from the reference checkout (.MISSING_LARGE_BLOBS), but its .mtl and
its six 1024x1024 RGB diffuse PNGs are there; they are committed under tests/golden/objects/ as data.
The reference's loader never sets has_texcoords (asset_utils/types.h:105), so every vertex uv is (0,0)
and TriangleToSupportedMat's texture() (raytrace_utils.glsl:140-175) reads the bilinear mix of the four
corner texels (GL_REPEAT, GL_LINEAR): body, wings and wing details 1.0, tail 0.62451 (159.25 / 255).
A stub OBJ gives each material one quad.  CPU: the host constant against those values and against an
independent numpy PNG decode.  GPU: the constant-albedo kernel and the per-hit TEX kernel render the
same frame, and both equal the oracle.
"""
import shutil
import struct
import zlib

import numpy as np
import pytest

import srt_amd as S
from conftest import GOLDEN, bits_equal, oracle_render

AIRPLANE = GOLDEN / "objects" / "11803_Airplane_v1_l1"
MATERIALS = ("11803_Airplane_body", "11803_Airplane_wing_R", "11803_Airplane_wing_details_R",
             "11803_Airplane_tail", "11803_Airplane_wing_details_L", "11803_Airplane_wing_L")
TEXTURE = {"11803_Airplane_body": "body", "11803_Airplane_wing_R": "wing_big_R",
           "11803_Airplane_wing_details_R": "wing_details_R", "11803_Airplane_tail": "tail",
           "11803_Airplane_wing_details_L": "wing_details_L", "11803_Airplane_wing_L": "wing_big_L"}
EXPECTED = {m: 1.0 for m in MATERIALS}
EXPECTED["11803_Airplane_tail"] = 0.62451  # SURVEY.md 8a TriangleToSupportedMat row / 8c item 5


def stub_obj(tmp_path):
    """The .mtl + PNGs next to an OBJ with one quad per material, facing the model camera."""
    for f in AIRPLANE.iterdir():
        shutil.copy(f, tmp_path / f.name)
    lines = ["mtllib 11803_Airplane_v1_l1.mtl"]
    for i, m in enumerate(MATERIALS):
        x0, x1 = -12.0 + 4.0 * i, -12.0 + 4.0 * i + 3.5
        lines += [f"v {x0} 2 0", f"v {x1} 2 0", f"v {x1} 16 0", f"v {x0} 16 0", f"usemtl {m}",
                  f"f {4 * i + 1} {4 * i + 2} {4 * i + 3} {4 * i + 4}"]
    lines += ["v -40 0 -20", "v 40 0 -20", "v 40 0 30", "v -40 0 30", "usemtl 11803_Airplane_wing_L", "f 25 26 27 28"]
    p = tmp_path / "airplane_stub.obj"
    p.write_text("\n".join(lines) + "\n")
    return p


def _png_rgb(path):
    """Independent decode of an 8-bit RGB, non-interlaced PNG (zlib + the five PNG filters)."""
    b = path.read_bytes()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w = 8, b"", None
    while pos < len(b):
        n = struct.unpack(">I", b[pos:pos + 4])[0]
        t = b[pos + 4:pos + 8]
        d = b[pos + 8:pos + 8 + n]
        if t == b"IHDR":
            w, h, bd, ct, _, _, il = struct.unpack(">IIBBBBB", d)
            assert bd == 8 and ct == 2 and il == 0
        elif t == b"IDAT":
            idat += d
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    out = np.zeros((h, 3 * w), np.int32)
    for y in range(h):
        f, line = raw[y, 0], raw[y, 1:].astype(np.int32)
        prev = out[y - 1] if y else np.zeros(3 * w, np.int32)
        cur = np.zeros(3 * w, np.int32)
        for x in range(3 * w):
            a = cur[x - 3] if x >= 3 else 0
            c = prev[x - 3] if x >= 3 else 0
            up = prev[x]
            if f == 0:
                p = 0
            elif f == 1:
                p = a
            elif f == 2:
                p = up
            elif f == 3:
                p = (a + up) // 2
            else:
                pa, pb, pc = abs(up - c), abs(a - c), abs(a + up - 2 * c)
                p = a if (pa <= pb and pa <= pc) else (up if pb <= pc else c)
            cur[x] = (line[x] + p) & 255
        out[y] = cur
    return out.reshape(h, w, 3).astype(np.uint8)


def _corner_mean(tex):
    """texture(sampler2D, (0,0)) under the sampling contract: x = y = -0.5, a = b = 0.5, texels (-1|0, -1|0)."""
    f = np.float32
    h, w, _ = tex.shape
    wt = f(0.5) * f(0.5)
    t = lambda i, j: tex[j, i].astype(np.float32) / f(255)  # noqa: E731
    return ((wt * t(w - 1, h - 1) + wt * t(0, h - 1)) + wt * t(w - 1, 0)) + wt * t(0, 0)


def test_airplane_uv0_albedo_host_constants(tmp_path):
    sc = S.Scene.from_models([S.load_obj(stub_obj(tmp_path))])
    assert (sc.mats["use_texture"][:6] == 1).all()
    for i, m in enumerate(MATERIALS):
        got = sc.tex_albedo[i]
        assert got[0] == got[1] == got[2]
        assert abs(float(got[0]) - EXPECTED[m]) < 1e-5, (m, got)
    assert sc.tex_albedo[3][0] == np.float32(159.25) / np.float32(255)  # tail: exactly the 4-corner mean
    # an independent decoder's corner texels give the same mix (body and tail: 1.0 and 159.25 / 255)
    for i, m in ((0, MATERIALS[0]), (3, MATERIALS[3])):
        tex = _png_rgb(tmp_path / f"11803_Airplane_{TEXTURE[m]}_diff.png")
        np.testing.assert_array_equal(_corner_mean(tex), sc.tex_albedo[i])


@pytest.mark.gpu
def test_airplane_uv0_albedo_gpu_constant_and_tex_kernels(tmp_path):
    from srt_amd import render as R
    from test_gpu_parity import gpu_render

    obj = stub_obj(tmp_path)
    const = R.make_setup(48, 40, show_model=True, models=[S.load_obj(obj)])
    sampled = R.make_setup(48, 40, show_model=True, models=[S.load_obj(obj, texcoords=True)])
    assert not const.scene.sample_textures and sampled.scene.sample_textures
    assert (sampled.scene.verts["uv"] == 0).all()  # no vt in the stub: every uv is (0,0), as in the reference
    a, o, _ = gpu_render(const, 3)
    b, p, _ = gpu_render(sampled, 3)
    assert bits_equal(a, b).all() and (o == p).all()
    want, want_o, _ = oracle_render(const, 3)
    assert bits_equal(a, want).all() and (o == want_o).all()
    want_s, _, _ = oracle_render(sampled, 3)
    assert bits_equal(b, want_s).all()
