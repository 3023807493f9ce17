"""Failure detection and checkpoint / resume on the GPU (SURVEY.md section 5 aux subsystems).

* NaN counter: accumulate_kernel counts path samples with a NaN component (the reference tests each
  sample for NaN and discards the result, raytrace_compute.glsl:408-410).  A light whose colour is NaN
  poisons every sample whose direct-light term selects it; the count is checked against the oracle's
  samples, each one recovered as the accumulation of one frame over a zero image.
* Checkpoint: srt_checkpoint_save / srt_checkpoint_load round trip, resumed frames bit-identical to an
  uninterrupted render, and the failure cases (other frame size or tiling, corrupt or missing file).
"""
from __future__ import annotations

import numpy as np
import pytest

import srt_amd as S
from srt_amd import render as R
from conftest import OBJECTS, bits_equal, oracle_render
from oracle import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rubik():
    return S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")


def _nan_light_setup(rubik, W=40, H=32):
    lights = list(S.MODEL_LIGHTS)
    lights[2] = S.PointLight((5.0, 15.0, 10.0), (float("nan"), 1.0, 0.2), 15.0)
    return R.make_setup(W, H, show_model=True, models=[rubik], lights=lights)


def _oracle_nan_samples(setup, spp):
    orc = O.Oracle(setup.scene, setup.lights, setup.noise, setup.noise_u)
    cam = setup.camera
    n = 0
    for k in range(2, spp + 2):  # frame k's samples: one frame accumulated over zeros
        f = O.Oracle.frame(setup.width, setup.height, accum_frames=k, show_model=True, bvh_count=setup.bvh_count,
                           light_count=len(setup.lights), max_depth=setup.max_depth, origin=cam.position,
                           direction=cam.front, up=cam.up, right=cam.right)
        acc = np.zeros((setup.height, setup.width, 4), np.float32)
        out = np.zeros((setup.height, setup.width, 4), np.uint8)
        orc.dispatch(f, acc, out)
        n += int(np.isnan(acc[..., :3]).any(axis=-1).sum())
    return n


def test_nan_samples_counted(rubik):
    setup = _nan_light_setup(rubik)
    spp = 4
    want = _oracle_nan_samples(setup, spp)
    assert want > 0
    want_acc, _, _ = oracle_render(setup, spp)
    r = R.Renderer(setup)
    try:
        assert r.compute.nan_samples() == 0
        r.render(spp)
        r.finish()
        assert bits_equal(r.accum(), want_acc).all()
        assert r.compute.nan_samples() == want
        r.render(spp)  # cumulative until reset_stats
        assert r.compute.nan_samples() == 2 * want
        r.compute.reset_stats()
        assert r.compute.nan_samples() == 0
    finally:
        r.close()
    clean = R.make_setup(40, 32, show_model=True, models=[rubik])
    r = R.Renderer(clean)
    try:
        r.render(spp)
        assert r.compute.nan_samples() == 0
    finally:
        r.close()


def test_bounce_cap_counted_apart_from_stack_overflow(rubik, monkeypatch):
    """Paths cut at the bounce cap have their own counter (srt_stats.bounce_cap), so an embedder can tell
    them from traversal stack overflows.  The reference's loop has no cap; the default (2^20) cuts nothing
    here and the frame is the oracle's, while SRT_BOUNCE_CAP=2 cuts every path still alive after two
    bounces and counts them, with no stack overflow."""
    setup = R.make_setup(40, 32, show_model=True, models=[rubik], max_depth=8)
    want_acc, _, want_st = oracle_render(setup, 2)
    r = R.Renderer(setup)
    try:
        r.render(2, count=True)
        r.finish()
        st = r.compute.stats()
        assert bits_equal(r.accum(), want_acc).all()
        assert st["bounce_cap"] == 0 and st["stack_overflow"] == 0
    finally:
        r.close()
    monkeypatch.setenv("SRT_BOUNCE_CAP", "2")
    r = R.Renderer(setup)
    try:
        r.render(2, count=True)
        r.finish()
        st = r.compute.stats()
        assert st["bounce_cap"] > 0 and st["stack_overflow"] == 0
        assert st["rays"] < want_st["rays"]
        assert not bits_equal(r.accum(), want_acc).all()
    finally:
        r.close()


def test_checkpoint_resume_is_bit_identical(rubik, tmp_path):
    setup = R.make_setup(48, 40, show_model=True, models=[rubik])
    want_acc, want_out, _ = oracle_render(setup, 5)
    ck = tmp_path / "run.ckpt"
    r = R.Renderer(setup)
    try:
        r.render(3)
        r.finish()
        r.compute.checkpoint_save(ck)
    finally:
        r.close()
    r = R.Renderer(setup)  # a fresh context, as after a restart
    try:
        af = r.compute.checkpoint_load(ck)
        assert af == 4  # the reset frame + 3 sampled frames
        r.accum_frames = af
        r.render(2, clear=False)
        r.finish()
        assert bits_equal(r.accum(), want_acc).all() and (r.output() == want_out).all()
        # another frame size or tiling is refused; a corrupt or missing file is an I/O error
        c = r.compute
        blob = bytearray(ck.read_bytes())
        blob[-5] ^= 0x40
        bad = tmp_path / "bad.ckpt"
        bad.write_bytes(bytes(blob))
        with pytest.raises(S.SrtError) as e:
            c.checkpoint_load(bad)
        assert e.value.code == S._lib.SRT_ERR_IO
        with pytest.raises(S.SrtError) as e:
            c.checkpoint_load(tmp_path / "missing.ckpt")
        assert e.value.code == S._lib.SRT_ERR_IO
        (tmp_path / "short.ckpt").write_bytes(ck.read_bytes()[:100])
        with pytest.raises(S.SrtError) as e:
            c.checkpoint_load(tmp_path / "short.ckpt")
        assert e.value.code == S._lib.SRT_ERR_IO
    finally:
        r.close()
    other = R.Renderer(R.make_setup(40, 40, show_model=True, models=[rubik]))
    try:
        with pytest.raises(S.SrtError) as e:
            other.compute.checkpoint_load(ck)
        assert e.value.code == S._lib.SRT_ERR_INVALID
    finally:
        other.close()
    banded = R.Renderer(setup, rank=0, nranks=2, band_rows=8)
    try:
        with pytest.raises(S.SrtError) as e:
            banded.compute.checkpoint_load(ck)
        assert e.value.code == S._lib.SRT_ERR_INVALID
    finally:
        banded.close()
