"""The multi-GPU frame through the C ABI (srt_group_*, include/srt_amd.h): a C++ host tiles the frame over
the devices of one process, as src/main.cpp:657-725's loop would over 8 GPUs.

On the one-GPU box: a group of one context gathers through RCCL (ncclGather, one communicator); groups of
2-4 contexts on the same device gather through device copies (RCCL takes one rank per device).  Every
group's assembled frame must be the one-context frame bit for bit, and the oracle's."""
from __future__ import annotations

import pytest

import srt_amd as S
from srt_amd import render as R
from conftest import OBJECTS, bits_equal, oracle_render

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    return R.make_setup(64, 48, show_model=True, models=[S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")])


@pytest.fixture(scope="module")
def want(setup):
    return oracle_render(setup, 3)


def _group_frame(setup, devices, band_rows, per_frame=False, spp=3):
    g = R.GroupRenderer(setup, devices, band_rows=band_rows)
    try:
        if per_frame:
            g.clear()
            for _ in range(spp):
                g.frame()
        else:
            g.render(spp)
        g.finish()
        return g.accum(), g.output(), g.transport
    finally:
        g.close()


def test_group_of_one_gathers_over_rccl(setup, want):
    acc, out, transport = _group_frame(setup, [0], 8)
    assert transport == "rccl"
    assert bits_equal(acc, want[0]).all() and (out == want[1]).all()


@pytest.mark.parametrize("n,band_rows", [(2, 8), (3, 2), (4, 1), (8, 8)])
def test_group_on_one_device_copies(setup, want, n, band_rows):
    acc, out, transport = _group_frame(setup, [0] * n, band_rows)
    assert transport == "copy"
    assert bits_equal(acc, want[0]).all() and (out == want[1]).all()


def test_group_per_frame_dispatch(setup, want):
    """srt_group_dispatch per frame (reset frame + 3 sampled frames) gives the fused render's frame."""
    acc, out, _ = _group_frame(setup, [0, 0], 8, per_frame=True)
    assert bits_equal(acc, want[0]).all() and (out == want[1]).all()


def test_group_forced_copy_transport(setup, want, monkeypatch):
    monkeypatch.setenv("SRT_GROUP_TRANSPORT", "copy")
    acc, out, transport = _group_frame(setup, [0], 8)
    assert transport == "copy"
    assert bits_equal(acc, want[0]).all() and (out == want[1]).all()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_cpp_compute_group_main_loop(setup, want, tmp_path, devices):
    """src/main.cpp's loop over Graphics::ComputeGroup (the C++ mirror, include/srt/srt.hpp): reset frame +
    3 dispatches, tiled over the listed devices and gathered to the first; the frame is the oracle's."""
    import subprocess

    import numpy as np

    from conftest import PKG, ROOT

    exe = ROOT / "tests" / "cpp" / "_build" / "test_group"
    exe.parent.mkdir(exist_ok=True)
    if not exe.exists():
        subprocess.run(["g++", "-std=c++17", "-O1", "-I", str(ROOT / "include"), str(ROOT / "tests/cpp/test_group.cpp"),
                        "-o", str(exe), "-L", str(PKG), "-lsrt_amd", f"-Wl,-rpath,{PKG}"], check=True)
    shaders = tmp_path / "shaders"
    shaders.mkdir()
    (shaders / "raytrace_compute.glsl").write_text("#version 450\n")
    res = subprocess.run([str(exe), str(OBJECTS) + "/", str(shaders) + "/", str(tmp_path / "g"), "8"]
                         + [str(d) for d in devices], capture_output=True, text=True, timeout=120)
    last = res.stdout.strip().splitlines()[-1] if res.stdout.strip() else ""  # (RCCL prints a banner first)
    assert res.returncode == 0 and last.startswith("OK"), res.stdout + res.stderr
    assert last.split()[1] == ("rccl" if len(set(devices)) == len(devices) else "copy")
    acc = np.fromfile(tmp_path / "g.accum", np.float32).reshape(48, 64, 4)
    out = np.fromfile(tmp_path / "g.rgba8", np.uint8).reshape(48, 64, 4)
    assert bits_equal(acc, want[0]).all() and (out == want[1]).all()
