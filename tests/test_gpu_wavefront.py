"""GPU parity of wavefront mode (wavefront.hpp): global-scene launches through wf_logic / wf_shade /
wf_trace render the oracle's frame bit for bit, with the counting instance of sample_kernel's CheckHit
counts (gpu_render renders the counting launch, then the timed launch through wavefront mode, and the two
frames must match)."""
import numpy as np
import pytest

import srt_amd as S
from srt_amd import render as R
from conftest import OBJECTS, bits_equal
from test_gpu_parity import assert_parity, gpu_render

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rubik():
    return S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")


@pytest.fixture
def wavefront(monkeypatch):
    monkeypatch.setenv("SRT_WAVEFRONT", "1")
    return monkeypatch


@pytest.mark.parametrize("env", [{}, {"SRT_WF_SLOTS": "300"}, {"SRT_WF_SLOTS": "5000", "SRT_WF_WAVES": "4"},
                                 {"SRT_GLOBAL_FUSED_MODE": "0", "SRT_NODE_ALIGN": "1"},
                                 {"SRT_WF_WAVES": "8", "SRT_NODE_LAYOUT": "0"},
                                 {"SRT_WF_WAVES": "5", "SRT_TRAV_FRAC16_GLOBAL": "16"}])
def test_wavefront_synthetic(wavefront, env):
    """Two synthetic soups (the second moved), every trace instance and layout, slot pools far smaller
    than the frame (many refills per slot) and larger."""
    for k, v in env.items():
        wavefront.setenv(k, v)
    assert_parity(R.make_setup(48, 40, show_model=True, models=[R.synthetic_model(30000, seed=3)]), 2)
    two = R.make_setup(40, 32, show_model=True, models=[R.synthetic_model(20000, seed=4),
                                                        R.synthetic_model(5000, seed=6)])
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (1.5, -2.0, 0.5)
    two.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(two, 2)


@pytest.mark.parametrize("w,h,spp,depth", [(64, 48, 3, 5), (33, 17, 2, 0), (40, 72, 2, 8)])
def test_wavefront_rubik_global(rubik, wavefront, w, h, spp, depth):
    wavefront.setenv("SRT_FORCE_GLOBAL_SCENE", "1")
    wavefront.setenv("SRT_WF_SLOTS", "1000")
    assert_parity(R.make_setup(w, h, show_model=True, models=[rubik], max_depth=depth), spp)


def test_wavefront_surface_mesh(wavefront):
    assert_parity(R.make_setup(64, 40, show_model=True, models=[R.torus_knot_model()]), 2)


def test_wavefront_per_frame_and_tiling(rubik, wavefront):
    """Per-frame dispatches and a 3-rank row-band split go through wavefront mode too."""
    wavefront.setenv("SRT_FORCE_GLOBAL_SCENE", "1")
    setup = R.make_setup(48, 40, show_model=True, models=[rubik])
    acc, out = assert_parity(setup, 3)
    acc_d, out_d, _ = gpu_render(setup, 3, per_frame=True)
    assert bits_equal(acc_d, acc).all() and (out_d == out).all()
    parts = [gpu_render(setup, 3, rank=r, nranks=3, band_rows=8)[0] for r in range(3)]
    from srt_amd import parallel as PAR

    rows_pad = PAR.rows_pad(40, 8, 3)
    stacked = np.zeros((3, rows_pad, 48, 4), np.float32)
    for r, p in enumerate(parts):
        stacked[r, :len(p)] = p
    assert bits_equal(PAR.assemble_host(stacked, 40, 8), acc).all()


def test_wavefront_sampled_textures(tmp_path, wavefront):
    """The texture-sampling shading instance (wf_shade_kernel<true>), two models with a transform."""
    from test_gpu_parity import _textured_obj

    obj = _textured_obj(tmp_path)
    wavefront.setenv("SRT_FORCE_GLOBAL_SCENE", "1")
    setup = R.make_setup(48, 40, show_model=True, models=[S.load_obj(obj, texcoords=True),
                                                          S.load_obj(obj, texcoords=True)], bvh_count=3)
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (4.0, -3.0, 7.0)
    setup.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(setup, 2)


@pytest.mark.parametrize("env", [{"SRT_TREELET_DEPTH": "3"}, {"SRT_TREELET_DEPTH": "6", "SRT_WF_SLOTS": "700"},
                                 {"SRT_TREELET_DEPTH": "9", "SRT_GLOBAL_FUSED_MODE": "0", "SRT_NODE_ALIGN": "1"},
                                 {"SRT_TREELET_DEPTH": "5", "SRT_NODE_LAYOUT": "0", "SRT_WF_WAVES": "4"},
                                 {"SRT_TREELET_DEPTH": "1", "SRT_GLOBAL_FUSED_MODE": "1"},
                                 {"SRT_TREELET_DEPTH": "4", "SRT_WF_SLOTS": "100000", "SRT_WF_WAVES": "8"}])
def test_treelets_synthetic(wavefront, env):
    """Treelet scheduling of the trace stage (rays suspended at treelet roots by wf_top_kernel, walked
    through their treelet by wf_bottom_kernel, resumed at the next pop): every treelet depth, layout and
    schedule renders the oracle's frame, two models (the second moved) included."""
    wavefront.setenv("SRT_TREELETS", "1")
    for k, v in env.items():
        wavefront.setenv(k, v)
    setup = R.make_setup(48, 40, show_model=True, models=[R.synthetic_model(30000, seed=3)])
    r = R.Renderer(setup)
    try:
        assert r.compute.GetInt("scene.treelets") > 0
    finally:
        r.close()
    assert_parity(setup, 2)
    two = R.make_setup(40, 32, show_model=True, models=[R.synthetic_model(20000, seed=4),
                                                        R.synthetic_model(5000, seed=6)])
    frame = np.eye(4, dtype=np.float32)
    frame[3, :3] = (1.5, -2.0, 0.5)
    two.scene.bvhs[1]["frame"] = frame.reshape(16)
    assert_parity(two, 2)


@pytest.mark.parametrize("depth", ["2", "4", "7"])
def test_treelets_rubik_and_surface(rubik, wavefront, depth):
    wavefront.setenv("SRT_TREELETS", "1")
    wavefront.setenv("SRT_TREELET_DEPTH", depth)
    wavefront.setenv("SRT_FORCE_GLOBAL_SCENE", "1")
    assert_parity(R.make_setup(64, 48, show_model=True, models=[rubik]), 3)
    assert_parity(R.make_setup(48, 40, show_model=True, models=[R.torus_knot_model()]), 2)
