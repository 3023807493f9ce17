"""Interactive mode: Camera::MoveAndRotate, Move*, Rotate, Reset
(src/raytracer/camera.cpp:71-212) and the frame loop's accumulation-reset schedule
(src/main.cpp:622-659), checked frame by frame against the oracle's restatement
(oracle/scene_ref.py CameraRef), and on the GPU a 240-frame scripted session
rendered through the C ABI against the oracle's per-frame dispatches.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import srt_amd as S
from srt_amd import _lib
from camera_script import camera_script
from conftest import OBJECTS, bits_equal
from oracle import scene_ref as REF


def _state(cam: S.Camera):
    return (cam.position.tobytes(), cam.front.tobytes(), cam.up.tobytes(), cam.right.tobytes(),
            np.float32(cam.yaw).tobytes(), np.float32(cam.pitch).tobytes(), cam.state.frame_counter)


def _state_ref(c: REF.CameraRef):
    v = lambda t: np.array(t, np.float32).tobytes()  # noqa: E731
    return (v(c.position), v(c.front), v(c.up), v(c.right), np.float32(c.yaw).tobytes(),
            np.float32(c.pitch).tobytes(), c.frame_counter)


def run_session(show_model: bool, script, on_frame=None):
    """Drive srt_progressive_frame and the oracle's restatement side by side; `on_frame(i, cam, accum_frames,
    reset)` runs after each frame's host step (the caller dispatches there)."""
    cam, ref = S.Camera(show_model), REF.CameraRef(show_model)
    assert _state(cam) == _state_ref(ref)
    inp = S.InputState()          # the app starts with the reset flag up (main.cpp:451)
    ref_flag, af, ref_af = True, 0, 0
    resets = 0
    for i, fr in enumerate(script):
        if fr.key == "R":         # KeyCallback GLFW_KEY_R (input_handler.cpp:56-61)
            cam.Reset()
            ref.reset()
            inp.should_reset_buffer = ref_flag = True
        elif fr.key == "L":
            inp.should_reset_buffer = ref_flag = True
        inp.movement_delta, inp.rotation_delta, inp.mouse_left = fr.move, fr.rot, fr.mouse_left
        af, reset = S.progressive_frame(cam, inp, fr.dt, af)
        ref_af, ref_reset, ref_flag = REF.progressive_frame_ref(ref, fr.move, fr.rot, fr.mouse_left, ref_flag,
                                                                fr.dt, ref_af)
        assert (af, reset, inp.should_reset_buffer) == (ref_af, ref_reset, ref_flag), i
        assert _state(cam) == _state_ref(ref), i
        resets += reset
        if on_frame is not None:
            on_frame(i, cam, af, reset)
    return cam, resets


@pytest.mark.parametrize("show_model", [True, False])
def test_scripted_session_matches_restatement(show_model):
    script = camera_script()
    cam, resets = run_session(show_model, script)
    assert cam.state.frame_counter == 240 and 20 < resets < 200
    assert -180.0 <= cam.yaw <= 180.0


def test_yaw_wrap_and_pitch_clamp():
    cam, ref = S.Camera(True), REF.CameraRef(True)
    for rot in ((170.0, 95.0), (400.0, -300.0), (-1000.0, 0.5), (0.00005, 0.0), (0.0, -0.00011)):
        cam.MoveAndRotate(0.016, (0.0, 0.0, 0.0), rot, 1.0)
        ref.move_and_rotate(0.016, (0.0, 0.0, 0.0), rot, 1.0)
        assert _state(cam) == _state_ref(ref)
        assert -180.0 <= cam.yaw <= 180.0 and -89.0 <= cam.pitch <= 89.0
    # a yaw the reference's wrap loop could never bring into range is refused, camera unchanged
    before = _state(cam)
    for bad in (float("inf"), 3.0e38):
        with pytest.raises(S.SrtError):
            cam.MoveAndRotate(0.016, (0.0, 0.0, 0.0), (bad, 0.0), 1.0)
        assert _state(cam) == before


def test_move_rotate_reset_calls():
    cam, ref = S.Camera(False), REF.CameraRef(False)
    steps = [("move", d, 0.37 * (d + 1)) for d in range(6)] + [("rot", 33.0, 120.0), ("rot", -500.0, -300.0)]
    for kind, a, b in steps:
        if kind == "move":
            getattr(cam, ("MoveForward", "MoveBackward", "MoveLeft", "MoveRight", "MoveUp", "MoveDown")[a])(b)
            ref.move(a, b)
        else:
            cam.Rotate(a, b)
            ref.rotate(a, b)
        assert _state(cam) == _state_ref(ref)
    assert cam.pitch == -89.0 and cam.yaw < -180.0  # Rotate clamps pitch but never wraps yaw
    cam.Reset()
    ref.reset()
    assert _state(cam) == _state_ref(ref)
    assert cam.position.tolist() == [0.0, 1.0, 4.0]
    with pytest.raises(S.SrtError):
        _lib.check(_lib.lib().srt_camera_move(C.byref(cam.state), 6, C.c_float(1.0)), "srt_camera_move")


def test_reorthonormalisation_every_120th_call():
    """camera.cpp:173-184: the basis is rebuilt from front on calls 120, 240, ... even with no input."""
    cam, ref = S.Camera(True), REF.CameraRef(True)
    for i in range(1, 241):
        cam.MoveAndRotate(0.01, (0.0, 0.0, 0.0), (0.0, 0.0), 1.0)
        ref.move_and_rotate(0.01, (0.0, 0.0, 0.0), (0.0, 0.0), 1.0)
        assert _state(cam) == _state_ref(ref)
    assert cam.state.frame_counter == 240


@pytest.mark.gpu
@pytest.mark.parametrize("show_model", [True, False])
def test_scripted_session_renders_oracle_frames(show_model):
    """240 frames of the scripted session, each one glDispatchCompute with the frame loop's uniforms
    (main.cpp:668-706), bit-exact against the oracle dispatching the same uniforms."""
    from oracle import pyoracle as O
    from srt_amd import render as R

    W, H = (32, 24) if show_model else (24, 16)
    models = [S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")] if show_model else None
    setup = R.make_setup(W, H, show_model=show_model, models=models)
    rdr = R.Renderer(setup, device=0)
    c = rdr.compute
    orc = O.Oracle(setup.scene, setup.lights, setup.noise, setup.noise_u)
    acc = np.zeros((H, W, 4), np.float32)
    out = np.zeros((H, W, 4), np.uint8)
    checked = []

    def on_frame(i, cam, accum_frames, reset):
        c.SetBool("resetAccumBuffer", reset)
        c.SetVec3("cameraOrigin", cam.getOrigin())
        c.SetVec3("cameraDirection", cam.getForward())
        c.SetVec3("cameraUp", cam.getUpVector())
        c.SetVec3("cameraRight", cam.getRightVector())
        c.SetInt("accumFrames", accum_frames)
        c.Dispatch((W + 7) // 8, (H + 7) // 8)
        f = O.Oracle.frame(W, H, show_model=show_model, bvh_count=setup.bvh_count, light_count=len(setup.lights),
                           max_depth=setup.max_depth, origin=cam.position, direction=cam.front, up=cam.up,
                           right=cam.right, accum_frames=accum_frames, reset=reset)
        orc.dispatch(f, acc, out)
        if i % 8 == 7 or i == 239:
            c.Finish()
            g_acc, g_out = c.read_accum(), c.read_output()
            assert bits_equal(g_acc, acc).all(), f"frame {i}: accumulation differs"
            assert (g_out == out).all(), f"frame {i}: image differs"
            checked.append(i)

    try:
        run_session(show_model, camera_script(), on_frame)
    finally:
        rdr.close()
    assert len(checked) == 30
