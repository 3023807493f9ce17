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


def test_group_serial_enqueue(setup, want, monkeypatch):
    """SRT_GROUP_THREADS=0: every context's launches enqueued from the calling thread (by default each
    context beyond the first has a launch thread of its own); the same frame."""
    monkeypatch.setenv("SRT_GROUP_THREADS", "0")
    acc, out, transport = _group_frame(setup, [0, 0, 0], 2, per_frame=True)
    assert transport == "copy"
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
    assert int(last.split()[2]) == len(devices)  # the ranks RCCL sees (or the contexts, copy transport)
    acc = np.fromfile(tmp_path / "g.accum", np.float32).reshape(48, 64, 4)
    out = np.fromfile(tmp_path / "g.rgba8", np.uint8).reshape(48, 64, 4)
    assert bits_equal(acc, want[0]).all() and (out == want[1]).all()


def _oracle_frames(setup, n):
    """The oracle's frame (accum, out) after each of n progressive dispatches (reset frame first)."""
    from oracle import pyoracle as O

    s = setup
    orc = O.Oracle(s.scene, s.lights, s.noise, s.noise_u)
    cam = s.camera
    f = O.Oracle.frame(s.width, s.height, show_model=s.show_model, bvh_count=s.bvh_count, light_count=len(s.lights),
                       max_depth=s.max_depth, origin=cam.position, direction=cam.front, up=cam.up, right=cam.right)
    import numpy as np

    acc = np.zeros((s.height, s.width, 4), np.float32)
    out = np.zeros((s.height, s.width, 4), np.uint8)
    f.reset, f.accum_frames = 1, 1
    orc.dispatch(f, acc, out)
    f.reset = 0
    frames = []
    for k in range(2, n + 2):
        orc.render(f, k, 1, acc, out)
        frames.append((acc.copy(), out.copy()))
    return frames


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_group_every_intermediate_frame(setup, devices):
    """srt_group_dispatch frame by frame, image0 read after every frame (the copy transport's
    write-after-read race could mix bands of frames N and N+1; the sRGB8 band images are now double-buffered
    with each render waiting for the gather that last read its buffer).  Every frame is the oracle's; only
    image0 crosses per frame, the radiance once, when it is read."""
    want = _oracle_frames(setup, 5)
    g = R.GroupRenderer(setup, devices, band_rows=8)
    try:
        g.clear()
        outs = []
        for _ in range(5):
            g.frame()
            outs.append(g.output())  # (finishes the group, then copies image0)
        assert g.get_int("gathers.output") == 5 and g.get_int("gathers.accum") == 0
        assert g.get_int("bytes.accum") == 4 * g.get_int("bytes.output")
        acc = g.accum()
        assert g.get_int("gathers.accum") == 1
        assert g.get_int("ranks") == len(devices)
    finally:
        g.close()
    for k, (wa, wo) in enumerate(want):
        assert (outs[k] == wo).all(), f"frame {k + 1}: image0 differs from the oracle's"
    assert bits_equal(acc, want[-1][0]).all()


def test_group_frames_back_to_back_without_reads(setup):
    """Five dispatches enqueued with no host sync between them (frame k's gather runs beside frame k+1's
    render on three contexts of one device), then one read: the oracle's frame."""
    want = _oracle_frames(setup, 5)[-1]
    g = R.GroupRenderer(setup, [0, 0, 0], band_rows=2)
    try:
        g.clear()
        for _ in range(5):
            g.frame()
        acc, out = g.accum(), g.output()
    finally:
        g.close()
    assert bits_equal(acc, want[0]).all() and (out == want[1]).all()


def test_group_destroy_detaches_contexts(setup, want):
    """srt_group_destroy detaches the caller's contexts from the freed band images without allocating
    (they kept pointers to the freed band images; VERDICT r04: the teardown allocated full-frame
    images on every context): rank 0 of 1 and no images, so a dispatch is refused with SRT_ERR_STATE; given
    images again (srt_alloc_images) each renders the whole frame."""
    import ctypes as C

    from srt_amd import _lib
    from srt_amd._lib import check, lib

    parts = [R.Renderer(setup) for _ in range(2)]
    try:
        ctxs = (C.c_void_p * 2)(*[p.compute.ctx for p in parts])
        g = C.c_void_p()
        check(lib().srt_group_create(ctxs, 2, 8, C.byref(g)), "group_create")
        check(lib().srt_group_alloc_images(g), "group_alloc_images")
        check(lib().srt_group_destroy(g), "group_destroy")
        for p in parts:
            assert p.compute.local_rows() == setup.height
            assert lib().srt_dispatch(p.compute.ctx, *p.groups) == _lib.SRT_ERR_STATE
            assert lib().srt_render_frames(p.compute.ctx, 2, 1, 1, 0) == _lib.SRT_ERR_STATE
            p.compute.alloc_images()
            p.render(3)
            p.finish()
            assert bits_equal(p.accum(), want[0]).all() and (p.output() == want[1]).all()
    finally:
        for p in parts:
            p.close()


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_group_kernel_and_exchange_time_back_to_back(setup, want, devices):
    """Group renders enqueued back to back with no finish between them (what bench.py's timed region does
    at N > 1): every context's sample launches are counted once, after the loop (srt_group_kernel_time),
    and so is each context's part of every frame's exchange (srt_group_exchange_time); the frame is the
    oracle's."""
    g = R.GroupRenderer(setup, devices, band_rows=8)
    try:
        g.render(3)
        g.finish()
        g.kernel_time(), g.exchange_time()  # drop the first render's
        for _ in range(4):
            g.render(3)  # (no finish)
        kt, ex = g.kernel_time(), g.exchange_time()
        assert [n for _, n in kt] == [4 * p.compute.GetInt("launch.chunks") for p in g.parts]
        assert all(ms > 0.0 for ms, _ in kt)
        assert [n for _, n in ex] == [4] * len(devices) and all(ms > 0.0 for ms, _ in ex)
        acc, out = g.accum(), g.output()
    finally:
        g.close()
    assert bits_equal(acc, want[0]).all() and (out == want[1]).all()


def test_bench_in_process_group_same_device(tmp_path):
    """`python bench.py --gpus 4 --same-device` without torch.distributed: the in-process device group
    (four contexts on GPU 0, device-copy transport) renders the one-GPU frame bit for bit, and the line
    names the transport, the ranks and every rank's kernel time; `--gpus 1 --group` runs the group with
    one RCCL rank (ncclCommInitAll, ncclGather) and renders the same frame."""
    import json
    import subprocess
    import sys

    import numpy as np

    from conftest import ROOT

    W, H, SPP = 96, 61, 3
    frames = {}
    lines = {}
    for n, extra in ((1, []), (4, ["--same-device"]), ("1g", ["--group"])):
        dump = tmp_path / f"f{n}.npz"
        cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(n)[0], "--steps", "2", "--warmup", "1",
               "--width", str(W), "--height", str(H), "--spp", str(SPP), "--band-rows", "2", "--no-cpu-baseline",
               "--no-global-leg", "--no-surface-leg", "--no-airplane-leg", "--dump", str(dump)] + extra
        env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        res = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env)
        assert res.returncode == 0, res.stderr[-3000:]
        lines[n] = json.loads([l for l in res.stdout.splitlines() if l.startswith("{")][-1])
        with np.load(dump) as z:
            frames[n] = (z["accum"], z["out"])
    assert bits_equal(frames[4][0], frames[1][0]).all() and (frames[4][1] == frames[1][1]).all()
    j = lines[4]
    assert j["n_gpus"] == 4 and j["value"] > 0
    assert j["group"]["transport"] == "copy" and j["group"]["rccl_ranks"] == 4 and j["group"]["contexts"] == 4
    assert len(j["kernel_ms_per_rank"]) == 4 and all(v > 0 for v in j["kernel_ms_per_rank"])
    # per rank: its render and its part of the exchange apart, and its share of the counted rays
    assert len(j["exchange_ms_per_rank"]) == 4 and all(v > 0 for v in j["exchange_ms_per_rank"])
    assert len(j["per_rank"]) == 4 and abs(sum(r["rays_share"] for r in j["per_rank"]) - 1.0) < 1e-3
    assert j["launch_overlap"] is True
    assert j["group"]["radiance_gathers_in_timed_steps"] == 0
    # --gpus 1 --group: the same in-process path with one RCCL rank (what N > 1 runs on distinct devices)
    g = lines["1g"]
    assert g["group"]["transport"] == "rccl" and g["group"]["rccl_ranks"] == 1
    assert bits_equal(frames["1g"][0], frames[1][0]).all() and (frames["1g"][1] == frames[1][1]).all()


def test_bench_group_of_one_agrees_with_single(tmp_path):
    """`--gpus 1 --group` (the in-process group's code path with one RCCL rank: back-to-back steps, the
    per-frame gather and assembly) runs the metric frame through RCCL and reports its exchange.  How close its
    throughput is to the single-context line is a measurement, not a correctness property: it is
    reported as a warning and in gpurun_out/tests/group_of_one.json, never failed on, so one timing fluctuation
    cannot stop the parity suite (-x)."""
    import json
    import subprocess
    import sys
    import warnings

    from conftest import ROOT

    env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    vals = {}
    for name, extra in (("single", []), ("group", ["--group"])):
        cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--steps", "6", "--warmup", "1",
               "--no-cpu-baseline", "--no-global-leg", "--no-surface-leg", "--no-airplane-leg"] + extra
        res = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
        assert res.returncode == 0, res.stderr[-3000:]
        line = json.loads([l for l in res.stdout.splitlines() if l.startswith("{")][-1])
        vals[name] = line["value"]
        assert line["value"] > 0 and line["rays_per_step"] > 0
        if extra:
            assert line["group"]["transport"] == "rccl" and line["group"]["rccl_ranks"] == 1
            assert line["exchange_ms_per_rank"][0] > 0
    ratio = vals["group"] / vals["single"]
    out = ROOT / "gpurun_out" / "tests"
    out.mkdir(parents=True, exist_ok=True)
    (out / "group_of_one.json").write_text(json.dumps({**vals, "group_over_single": ratio}))
    if abs(ratio - 1.0) > 0.01:
        warnings.warn(f"group of one vs single context: {ratio:.4f} ({vals})")
