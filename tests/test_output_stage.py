"""Output stage: RGBA8 frames to PNG / PPM through the C ABI (CPU only).

The files are decoded here independently (zlib + the PNG chunk layout, the PPM header) and must
hold exactly the input bytes, rows flipped so that the kernel's bottom row (j = 0) comes last.
"""
import struct
import zlib

import numpy as np
import pytest

import srt_amd as S
from srt_amd import _lib


def _image(h=37, w=53, seed=4):
    return np.random.default_rng(seed).integers(0, 256, size=(h, w, 4), dtype=np.uint8)


def _read_png(path):
    data = path.read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, ihdr = 8, b"", None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body) & 0xFFFFFFFF
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype, _, _, interlace = ihdr
    assert (depth, ctype, interlace) == (8, 6, 0)
    raw = zlib.decompress(idat)
    rows = []
    for y in range(h):
        line = raw[y * (1 + 4 * w):(y + 1) * (1 + 4 * w)]
        assert line[0] == 0  # filter type None
        rows.append(np.frombuffer(line[1:], np.uint8).reshape(w, 4))
    return np.stack(rows)


def test_png_round_trip_flipped(tmp_path):
    img = _image()
    S.write_image(tmp_path / "f.png", img)
    assert (_read_png(tmp_path / "f.png") == img[::-1]).all()
    S.write_image(tmp_path / "g.PNG", img, flip_y=False)
    assert (_read_png(tmp_path / "g.PNG") == img).all()


def test_ppm_round_trip_drops_alpha(tmp_path):
    img = _image(9, 11)
    S.write_image(tmp_path / "f.ppm", img)
    data = (tmp_path / "f.ppm").read_bytes()
    header = b"P6\n11 9\n255\n"
    assert data.startswith(header)
    rgb = np.frombuffer(data[len(header):], np.uint8).reshape(9, 11, 3)
    assert (rgb == img[::-1, :, :3]).all()


def test_errors(tmp_path):
    img = _image(4, 4)
    with pytest.raises(S.SrtError) as e:
        S.write_image(tmp_path / "f.bmp", img)
    assert e.value.code == _lib.SRT_ERR_INVALID
    with pytest.raises(S.SrtError) as e:
        S.write_image(tmp_path / "missing_dir" / "f.png", img)
    assert e.value.code == _lib.SRT_ERR_IO
    with pytest.raises(ValueError):
        S.write_image(tmp_path / "f.png", img[..., :3])
