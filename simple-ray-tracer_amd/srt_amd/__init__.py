"""srt_amd -- MI355X-native path-tracing inner loop of matteobir12/simple-ray-tracer.

Host-side mirror of the reference's dispatch API for this path, over the C ABI
of ``libsrt_amd.so`` (include/srt_amd.h):

* :class:`Compute`          -- ``Graphics::Compute`` (include/graphics/shader.h:46-55):
                               ``Init/Use/SetBool/SetInt/SetUInt/SetFloat/SetVec3`` +
                               ``Dispatch`` (``glDispatchCompute``) and ``Finish`` (``glFinish``).
* :func:`LoadObject`        -- ``AssetUtils::LoadObject`` (src/asset_utils/model_loader.cpp:20-32).
* :func:`UploadModelDataToGPU` / :func:`UpdateModelMatrix`
                            -- src/asset_utils/gpu_loader.cpp:63-196.
* :class:`Camera`, :class:`PointLight`, :func:`generate_noise`
                            -- the per-frame inputs src/main.cpp feeds the kernel.

Everything computes through the HIP kernels; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import pathlib
import sys
from dataclasses import dataclass, field
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from ._lib import SrtError, check, lib

__all__ = [
    "Compute", "Model", "Scene", "LoadObject", "load_obj", "model_from_triangles", "UploadModelDataToGPU",
    "UpdateModelMatrix", "Camera", "InputState", "progressive_frame", "PointLight", "generate_noise", "glibc_rand", "SrtError",
    "NODE_DTYPE", "BVH_DTYPE", "MAT_DTYPE", "TRI_DTYPE", "VERT_DTYPE", "LIGHT_DTYPE", "RAY_DTYPE",
    "MODEL_LIGHTS", "SPHERE_LIGHTS", "REFERENCE_OBJECTS",
]

# std430 record layouts (include/srt_amd.h == gpu_loader.cpp:11-41)
BVH_DTYPE = np.dtype([("first_index", "<u4"), ("count", "<u4"), ("pad", "<u4", 2), ("frame", "<f4", 16)])
NODE_DTYPE = np.dtype([("min", "<f4", 3), ("first", "<u4"), ("max", "<f4", 3), ("count", "<u4")])
MAT_DTYPE = np.dtype([("diffuse", "<f4", 3), ("Ns", "<f4"), ("Ks", "<f4", 3), ("use_texture", "<u4"),
                      ("handle", "<u4", 2), ("pad", "<u4", 2)])
TRI_DTYPE = np.dtype([("v", "<u4", 3), ("mat", "<u4")])
VERT_DTYPE = np.dtype([("pos", "<f4", 3), ("pad0", "<f4"), ("uv", "<f4", 2), ("pad1", "<f4", 2)])
LIGHT_DTYPE = np.dtype([("pos", "<f4", 3), ("intensity", "<f4"), ("color", "<f4", 3), ("pad", "<f4")])
RAY_DTYPE = np.dtype([("o", "<f4", 3), ("pad", "<f4"), ("d", "<f4", 3), ("t", "<f4")])
for _dt, _n in ((BVH_DTYPE, 80), (NODE_DTYPE, 32), (MAT_DTYPE, 48), (TRI_DTYPE, 16), (VERT_DTYPE, 32),
                (LIGHT_DTYPE, 32), (RAY_DTYPE, 32)):
    assert _dt.itemsize == _n

# The reference checkout's assets are not shipped; callers point at a copy.
REFERENCE_OBJECTS = pathlib.Path("/root/reference/objects")


def _ptr(a: np.ndarray | None):
    return None if a is None else C.c_void_p(a.ctypes.data)


# ---------------------------------------------------------------------------
# camera / lights / noise (the inputs src/main.cpp produces)
# ---------------------------------------------------------------------------
@dataclass
class PointLight:
    """RayTracer::PointLight (include/raytracer/light.h:54-63)."""
    position: Sequence[float]
    color: Sequence[float]
    intensity: float


# src/main.cpp:584-589 (model scene) and :593-594 (sphere scene)
MODEL_LIGHTS = (
    PointLight((1.0, 10.0, 10.0), (1.0, 1.0, 1.0), 50.0),
    PointLight((-5.0, 15.0, 10.0), (1.0, 0.2, 0.2), 15.0),
    PointLight((5.0, 15.0, 10.0), (0.2, 1.0, 0.2), 15.0),
    PointLight((-5.0, 5.0, 10.0), (0.2, 0.2, 1.0), 15.0),
    PointLight((5.0, 5.0, 10.0), (1.0, 1.0, 0.1), 15.0),
    PointLight((0.0, 21.0, 17.0), (1.0, 1.0, 1.0), 50.0),
)
SPHERE_LIGHTS = (
    PointLight((1.0, 2.0, 0.0), (1.0, 1.0, 1.0), 10.0),
    PointLight((-2.5, 2.0, 0.0), (1.0, 1.0, 1.0), 3.0),
)


def lights_array(lights: Iterable[PointLight]) -> np.ndarray:
    ls = list(lights)
    a = np.zeros(len(ls), dtype=LIGHT_DTYPE)
    for i, l in enumerate(ls):
        a[i]["pos"] = np.asarray(l.position, dtype=np.float32)
        a[i]["color"] = np.asarray(l.color, dtype=np.float32)
        a[i]["intensity"] = np.float32(l.intensity)
    return a


class Camera:
    """RayTracer::Camera (src/raytracer/camera.cpp, include/raytracer/camera.h) over the C ABI's srt_camera
    state: construction + Initialize + Reset as src/main.cpp:439-441, Move*, Rotate, MoveAndRotate."""

    FORWARD, BACKWARD, LEFT, RIGHT, UP, DOWN = range(6)

    def __init__(self, show_model: bool = True):
        self.show_model = bool(show_model)
        self.state = _lib.CameraState()
        check(lib().srt_camera_init(C.byref(self.state), int(self.show_model)), "srt_camera_init")

    def Reset(self):
        check(lib().srt_camera_state_reset(C.byref(self.state)), "srt_camera_state_reset")

    def Rotate(self, yaw_offset: float, pitch_offset: float):
        check(lib().srt_camera_rotate(C.byref(self.state), C.c_float(yaw_offset), C.c_float(pitch_offset)),
              "srt_camera_rotate")

    def _move(self, direction: int, delta: float):
        check(lib().srt_camera_move(C.byref(self.state), direction, C.c_float(delta)), "srt_camera_move")

    def MoveForward(self, delta: float):
        self._move(self.FORWARD, delta)

    def MoveBackward(self, delta: float):
        self._move(self.BACKWARD, delta)

    def MoveLeft(self, delta: float):
        self._move(self.LEFT, delta)

    def MoveRight(self, delta: float):
        self._move(self.RIGHT, delta)

    def MoveUp(self, delta: float):
        self._move(self.UP, delta)

    def MoveDown(self, delta: float):
        self._move(self.DOWN, delta)

    def MoveAndRotate(self, delta_time: float, movement_delta, rotation_delta, movement_speed: float):
        m = np.asarray(movement_delta, np.float32).reshape(3)
        r = np.asarray(rotation_delta, np.float32).reshape(2)
        check(lib().srt_camera_move_and_rotate(C.byref(self.state), C.c_float(delta_time), _ptr(m), _ptr(r),
                                               C.c_float(movement_speed)), "srt_camera_move_and_rotate")

    def _v(self, name):
        return np.array(getattr(self.state, name)[:], np.float32)

    @property
    def position(self):
        return self._v("position")

    @position.setter
    def position(self, v):
        self.state.position[:] = [float(x) for x in np.asarray(v, np.float32).reshape(3)]

    @property
    def front(self):
        return self._v("front")

    @property
    def up(self):
        return self._v("up")

    @property
    def right(self):
        return self._v("right")

    @property
    def yaw(self):
        return np.float32(self.state.yaw)

    @property
    def pitch(self):
        return np.float32(self.state.pitch)

    def getOrigin(self):
        return self.position

    def getForward(self):
        return self.front

    def getUpVector(self):
        return self.up

    def getRightVector(self):
        return self.right


@dataclass
class InputState:
    """What the frame loop reads from InputHandler each frame (include/input_handler.h): the movement and
    rotation deltas, the left mouse button, and the handler's shouldResetBuffer flag.  The app starts with the
    flag up (EnableMouseCapture(false), src/main.cpp:451, input_handler.cpp:172)."""
    movement_delta: Sequence[float] = (0.0, 0.0, 0.0)
    rotation_delta: Sequence[float] = (0.0, 0.0)
    mouse_left: bool = False
    should_reset_buffer: bool = True


def progressive_frame(camera: Camera, inp: InputState, delta_time: float, accum_frames: int) -> tuple[int, bool]:
    """One frame of src/main.cpp:622-659: returns (accumFrames, resetAccumBuffer) to upload; moves the camera
    and clears inp.should_reset_buffer as the loop does."""
    m = np.asarray(inp.movement_delta, np.float32).reshape(3)
    r = np.asarray(inp.rotation_delta, np.float32).reshape(2)
    flag = C.c_int32(int(bool(inp.should_reset_buffer)))
    af = C.c_int32(int(accum_frames))
    reset = C.c_int32(0)
    check(lib().srt_progressive_frame(C.byref(camera.state), _ptr(m), _ptr(r), int(bool(inp.mouse_left)),
                                      C.byref(flag), C.c_float(delta_time), C.byref(af), C.byref(reset)),
          "srt_progressive_frame")
    inp.should_reset_buffer = bool(flag.value)
    return int(af.value), bool(reset.value)


def glibc_rand(n: int) -> np.ndarray:
    out = np.zeros(n, np.int32)
    check(lib().srt_glibc_rand(n, _ptr(out)), "srt_glibc_rand")
    return out


def write_image(path: str | pathlib.Path, rgba8: np.ndarray, flip_y: bool = True) -> None:
    """Output stage (replaces the GL display quad, src/main.cpp:303-349): an (H, W, 4) uint8 image
    to PNG (RGBA) or binary PPM (RGB) by extension.  flip_y writes the kernel's bottom row last."""
    a = np.ascontiguousarray(rgba8, np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("write_image expects an (H, W, 4) uint8 array")
    check(lib().srt_image_write(str(path).encode(), _ptr(a), a.shape[1], a.shape[0], int(flip_y)), "srt_image_write")


def generate_noise(width: int, height: int, gcc_order: bool = True) -> tuple[np.ndarray, np.ndarray]:
    """UpdateNoiseTex (src/main.cpp:269-301): W*H unit vectors, then W*H uniform vec3s (RGB32F)."""
    texels = int(width) * int(height)
    noise = np.empty((texels, 3), np.float32)
    noise_u = np.empty((texels, 3), np.float32)
    check(lib().srt_noise_generate(texels, int(gcc_order), _ptr(noise), _ptr(noise_u)), "srt_noise_generate")
    return noise, noise_u


# ---------------------------------------------------------------------------
# models and scenes (host producers)
# ---------------------------------------------------------------------------
class Model:
    """AssetUtils::Model (include/asset_utils/types.h:39-52): BVH-ordered triangles + nodes."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)

    @property
    def handle(self):
        return self._h

    def info(self) -> dict:
        counts = np.zeros(8, np.uint64)
        mn = np.zeros(3, np.float32)
        mx = np.zeros(3, np.float32)
        check(lib().srt_model_info(self._h, _ptr(counts), _ptr(mn), _ptr(mx)), "srt_model_info")
        keys = ("triangles", "vertices", "nodes", "leaves", "max_depth", "materials", "faces_dropped")
        d = {k: int(counts[i]) for i, k in enumerate(keys)}
        d["root_min"], d["root_max"] = mn, mx
        return d

    def prim_order(self) -> np.ndarray:
        """The BVH's primitive permutation (bvh.h:66-72): GetPrims()[i] is loader triangle ``out[i]``."""
        sizes = np.zeros(4, np.uint32)
        check(lib().srt_model_sizes(self._h, _ptr(sizes)), "srt_model_sizes")
        out = np.zeros(sizes[1], np.uint32)
        check(lib().srt_model_prim_order(self._h, _ptr(out)), "srt_model_prim_order")
        return out

    def __del__(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.srt_model_free(self._h)
            self._h = None


SRT_LOAD_TEXCOORDS = 1


def load_obj(obj_path: str | pathlib.Path, texcoords: bool = False) -> Model:
    """LoadObject's parser on one .obj path.  ``texcoords=True`` gives vertices their ``vt`` uvs (the loader
    with has_texcoords set, model_loader.cpp:322-324); the reference leaves every uv at (0,0)."""
    h = C.c_void_p()
    flags = SRT_LOAD_TEXCOORDS if texcoords else 0
    check(lib().srt_model_load_ex(str(obj_path).encode(), flags, C.byref(h)), f"LoadObject({obj_path})")
    return Model(h.value)


def texture_sample(texels: np.ndarray, s: float, t: float) -> np.ndarray:
    """texture(sampler2D, vec2(s, t)).xyz on the host (the sampling contract);
    ``texels`` is (H, W, C) uint8, rows top first."""
    tex = np.ascontiguousarray(texels, np.uint8)
    if tex.ndim == 2:
        tex = tex[:, :, None]
    desc = _lib.Texture(tex.ctypes.data, tex.shape[1], tex.shape[0], tex.shape[2])
    out = np.zeros(3, np.float32)
    check(lib().srt_texture_sample(C.byref(desc), C.c_float(s), C.c_float(t), _ptr(out)), "texture_sample")
    return out


def LoadObject(name: str, objects_dir: str | pathlib.Path = "./objects/") -> Model:
    """AssetUtils::LoadObject(name): ``objects/<name>/<name>.obj`` (model_loader.cpp:20-32)."""
    return load_obj(pathlib.Path(objects_dir) / name / f"{name}.obj")


def model_from_triangles(xyz9: np.ndarray, kd=(0.8, 0.8, 0.8), ks=(0.0, 0.0, 0.0), ns: float = 10.0) -> Model:
    xyz9 = np.ascontiguousarray(xyz9, dtype=np.float32).reshape(-1, 9)
    kd = np.asarray(kd, np.float32)
    ks = np.asarray(ks, np.float32)
    h = C.c_void_p()
    check(lib().srt_model_from_triangles(_ptr(xyz9), xyz9.shape[0], _ptr(kd), _ptr(ks), C.c_float(ns), C.byref(h)),
          "srt_model_from_triangles")
    return Model(h.value)


@dataclass
class Scene:
    """The five SSBO arrays UploadModelDataToGPU builds (gpu_loader.cpp:44-52), std430 layouts."""
    bvhs: np.ndarray
    nodes: np.ndarray
    mats: np.ndarray
    tex_albedo: np.ndarray
    tris: np.ndarray
    verts: np.ndarray
    textures: list = field(default_factory=list)  # (H, W, C) uint8 per texture handle
    sample_textures: bool = False                  # sample at the hit's uv instead of tex_albedo
    tri_input: np.ndarray | None = None            # loader-order index of each triangle (srt_scene_tri_order)

    @classmethod
    def from_models(cls, models: Sequence[Model | None]) -> "Scene":
        hs = (C.c_void_p * max(len(models), 1))(*[(m.handle if m is not None else None) for m in models])
        sh = C.c_void_p()
        check(lib().srt_scene_build(hs, len(models), C.byref(sh)), "UploadModelDataToGPU")
        try:
            sizes = np.zeros(5, np.uint32)
            check(lib().srt_scene_sizes(sh, _ptr(sizes)), "srt_scene_sizes")
            s = cls(np.zeros(sizes[0], BVH_DTYPE), np.zeros(sizes[1], NODE_DTYPE), np.zeros(sizes[2], MAT_DTYPE),
                    np.zeros((sizes[2], 3), np.float32), np.zeros(sizes[3], TRI_DTYPE), np.zeros(sizes[4], VERT_DTYPE))
            check(lib().srt_scene_copy(sh, _ptr(s.bvhs), _ptr(s.nodes), _ptr(s.mats), _ptr(s.tex_albedo),
                                       _ptr(s.tris), _ptr(s.verts)), "srt_scene_copy")
            s.tri_input = np.zeros(sizes[3], np.uint32)
            check(lib().srt_scene_tri_order(sh, _ptr(s.tri_input)), "srt_scene_tri_order")
            n, sample = C.c_uint32(), C.c_int()
            check(lib().srt_scene_texture_count(sh, C.byref(n), C.byref(sample)), "srt_scene_texture_count")
            for i in range(n.value):
                t = _lib.Texture()
                check(lib().srt_scene_texture(sh, i, C.byref(t)), "srt_scene_texture")
                nbytes = t.width * t.height * t.channels
                buf = (C.c_uint8 * nbytes).from_address(t.texels)
                s.textures.append(np.frombuffer(buf, np.uint8).copy().reshape(t.height, t.width, t.channels))
            s.sample_textures = bool(sample.value)
        finally:
            lib().srt_scene_free(sh)
        return s


# ---------------------------------------------------------------------------
# Graphics::Compute
# ---------------------------------------------------------------------------
class Compute:
    """``Graphics::Compute`` backed by the HIP path tracer.

    ``path`` is accepted for interface parity with ``Compute(const char* path)``
    (Shader.cpp:14-26); the program is the built-in raytrace_compute kernel.
    ``stream`` is a hipStream_t handle (e.g. ``torch.cuda.current_stream().cuda_stream``).
    """

    def __init__(self, path: str | None = None, device: int = 0, stream: int | None = None):
        self.path = path
        self.device = device
        self._stream = stream
        self._ctx = None
        self.program = 0
        self.width = 0
        self.height = 0

    # -- lifecycle ----------------------------------------------------------
    def Init(self):
        if not getattr(self, "program", 0):
            # Compute::CreateComputeProgram (create_compute_program.h:46-72): 0 -> the reference terminates
            self.program = int(lib().srt_program_create((self.path or "builtin:raytrace_compute").encode()))
            if self.program == 0:
                raise RuntimeError(f"Compute::Init: no compute program for {self.path!r}: {_lib.last_error()}")
        if self._ctx is None:
            h = C.c_void_p()
            check(lib().srt_create(self.device, C.c_void_p(self._stream) if self._stream else None, C.byref(h)),
                  "Compute::Init")
            self._ctx = h
        return self

    def Use(self):
        self.Init()

    @property
    def ctx(self):
        if self._ctx is None:
            self.Init()
        return self._ctx

    def close(self):
        if self._ctx is not None:
            lib().srt_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            if self._ctx is not None and _lib._lib is not None:
                _lib._lib.srt_destroy(self._ctx)
                self._ctx = None
        except Exception:
            pass

    def __enter__(self):
        return self.Init()

    def __exit__(self, *exc):
        self.close()

    # -- uniforms (Shader.cpp:79-122, 159-212) ------------------------------
    def SetBool(self, name: str, val: bool):
        rc = lib().srt_set_bool(self.ctx, name.encode(), int(bool(val)))
        if rc == _lib.SRT_ERR_NOT_FOUND:
            if name != "resetAccumBuffer":  # Compute::SetBool's warning (Shader.cpp:170-176)
                print(f"Warning: Uniform '{name}' not found in compute shader", file=sys.stderr)
            return
        check(rc, f"SetBool({name})")

    def SetInt(self, name: str, val: int):
        rc = lib().srt_set_int(self.ctx, name.encode(), int(val))
        if rc == _lib.SRT_ERR_NOT_FOUND:  # silently ignored (Shader.cpp:190-205)
            return
        check(rc, f"SetInt({name})")
        if name == "Width":
            self.width = int(val)
        elif name == "Height":
            self.height = int(val)

    def GetInt(self, name: str) -> int:
        """An int / uint / bool uniform's value, or a scene choice: "scene.fused", "scene.global_waves",
        "scene.tri_slots" (srt_get_int)."""
        v = C.c_int()
        check(lib().srt_get_int(self.ctx, name.encode(), C.byref(v)), f"GetInt({name})")
        return v.value

    def SetUInt(self, name: str, val: int):
        rc = lib().srt_set_uint(self.ctx, name.encode(), int(val) & 0xFFFFFFFF)
        if rc != _lib.SRT_ERR_NOT_FOUND:
            check(rc, f"SetUInt({name})")

    def SetFloat(self, name: str, val: float):
        rc = lib().srt_set_float(self.ctx, name.encode(), float(val))
        if rc != _lib.SRT_ERR_NOT_FOUND:
            check(rc, f"SetFloat({name})")

    def SetVec3(self, name: str, val):
        v = np.asarray(val, dtype=np.float32).reshape(3)
        rc = lib().srt_set_vec3(self.ctx, name.encode(), float(v[0]), float(v[1]), float(v[2]))
        if rc != _lib.SRT_ERR_NOT_FOUND:
            check(rc, f"SetVec3({name})")

    # -- bindings ------------------------------------------------------------
    def bind_noise(self, noise: np.ndarray, noise_u: np.ndarray):
        noise = np.ascontiguousarray(noise, np.float32)
        noise_u = np.ascontiguousarray(noise_u, np.float32)
        if noise.shape != noise_u.shape or noise.ndim != 2 or noise.shape[1] != 3:
            raise ValueError("noise buffers must be (W*H, 3) float32")
        check(lib().srt_set_noise(self.ctx, _ptr(noise), _ptr(noise_u), noise.shape[0]), "bind_noise")

    def bind_lights(self, lights):
        arr = lights if isinstance(lights, np.ndarray) else lights_array(lights)
        arr = np.ascontiguousarray(arr, dtype=LIGHT_DTYPE)
        check(lib().srt_set_lights(self.ctx, _ptr(arr), len(arr)), "bind_lights")

    def bind_textures(self, textures: Sequence[np.ndarray]):
        """GPUTexture + GetHandle for each (H, W, C) uint8 texture: texture i gets handle i."""
        keep = [np.ascontiguousarray(t if t.ndim == 3 else t[:, :, None], np.uint8) for t in textures]
        descs = (_lib.Texture * max(len(keep), 1))(*[_lib.Texture(t.ctypes.data, t.shape[1], t.shape[0], t.shape[2])
                                                      for t in keep])
        check(lib().srt_upload_textures(self.ctx, descs, len(keep)), "bind_textures")

    def bind_scene(self, scene: Scene):
        s = scene
        if s.sample_textures:
            self.bind_textures(s.textures)
        tex = None if s.sample_textures else np.ascontiguousarray(s.tex_albedo, np.float32)
        check(lib().srt_upload_scene(self.ctx, _ptr(s.bvhs), len(s.bvhs), _ptr(s.nodes), len(s.nodes),
                                     _ptr(s.mats), _ptr(tex), len(s.mats), _ptr(s.tris), len(s.tris), _ptr(s.verts),
                                     len(s.verts)),
              "UploadModelDataToGPU")

    def set_tiling(self, rank: int, nranks: int, band_rows: int = 16):
        check(lib().srt_set_tiling(self.ctx, rank, nranks, band_rows), "set_tiling")

    def local_rows(self) -> int:
        return int(lib().srt_local_rows(self.ctx))

    def alloc_images(self):
        check(lib().srt_alloc_images(self.ctx), "alloc_images")

    def image_pointers(self) -> tuple[int, int]:
        a, o = C.c_void_p(), C.c_void_p()
        check(lib().srt_image_pointers(self.ctx, C.byref(a), C.byref(o)), "image_pointers")
        return a.value or 0, o.value or 0

    def set_image_buffers(self, accum_dev: int, out_dev: int):
        check(lib().srt_set_image_buffers(self.ctx, C.c_void_p(accum_dev), C.c_void_p(out_dev)), "set_image_buffers")

    def assemble_bands(self, gathered_dev: int, nranks: int, rows_pad: int, band_rows: int, frames: int,
                       accum_full_dev: int | None, out_full_dev: int | None):
        check(lib().srt_assemble_bands(self.ctx, C.c_void_p(gathered_dev), nranks, rows_pad, band_rows, frames,
                                       C.c_void_p(accum_full_dev) if accum_full_dev else None,
                                       C.c_void_p(out_full_dev) if out_full_dev else None), "assemble_bands")

    def assemble_output_bands(self, gathered_rgba8_dev: int, nranks: int, rows_pad: int, band_rows: int,
                              out_full_dev: int):
        """The per-frame root step: de-interleave the ranks' gathered sRGB8 rows into the full image0."""
        check(lib().srt_assemble_output_bands(self.ctx, C.c_void_p(gathered_rgba8_dev), nranks, rows_pad, band_rows,
                                              C.c_void_p(out_full_dev)), "assemble_output_bands")

    # -- dispatch -------------------------------------------------------------
    def Dispatch(self, groups_x: int, groups_y: int, groups_z: int = 1):
        """glDispatchCompute(groups_x, groups_y, 1) (src/main.cpp:706)."""
        if groups_z != 1:
            raise ValueError("the kernel is dispatched with groups_z == 1")
        check(lib().srt_dispatch(self.ctx, groups_x, groups_y), "Dispatch")

    def Finish(self):
        """glMemoryBarrier + glFinish (src/main.cpp:709-718)."""
        check(lib().srt_finish(self.ctx), "Finish")

    def render_frames(self, frame_first: int, nframes: int, write_output: bool = True, count: bool = False):
        check(lib().srt_render_frames(self.ctx, frame_first, nframes, int(write_output), int(count)),
              "render_frames")

    def stats(self) -> dict:
        """srt_get_stats, plus "shadow_rays" (srt_ray_kinds' shadow count, as the oracle's stats name it)."""
        s = _lib.Stats()
        check(lib().srt_get_stats(self.ctx, C.byref(s)), "stats")
        d = s.as_dict()
        d["shadow_rays"] = self.ray_kinds()["shadow"]
        return d

    def ray_kinds(self) -> dict:
        """The counted rays by kind (srt_ray_kinds): camera, shadow and bounce rays; they sum to stats()["rays"]."""
        k = np.zeros(3, np.uint64)
        check(lib().srt_ray_kinds(self.ctx, _ptr(k)), "ray_kinds")
        return {"camera": int(k[0]), "shadow": int(k[1]), "bounce": int(k[2])}

    def last_kernel_ms(self) -> float:
        """Device time of the sample-kernel launches of the last render (each launch's span on the GPU clock)."""
        ms = C.c_float()
        check(lib().srt_last_kernel_ms(self.ctx, C.byref(ms)), "last_kernel_ms")
        return float(ms.value)

    def kernel_time(self) -> tuple:
        """(summed kernel ms, launches) of the sample-kernel launches since the previous call."""
        ms, n = C.c_double(), C.c_int()
        check(lib().srt_kernel_time(self.ctx, C.byref(ms), C.byref(n)), "kernel_time")
        return float(ms.value), int(n.value)

    def reset_stats(self):
        check(lib().srt_reset_stats(self.ctx), "reset_stats")

    def nan_samples(self) -> int:
        """Path samples with a NaN component since creation / reset_stats (failure detection)."""
        v = C.c_uint64(0)
        check(lib().srt_nan_samples(self.ctx, C.byref(v)), "nan_samples")
        return int(v.value)

    def checkpoint_save(self, path):
        check(lib().srt_checkpoint_save(self.ctx, str(path).encode()), "checkpoint_save")

    def checkpoint_load(self, path) -> int:
        """Restores the accumulation image, accumFrames and the camera uniforms; returns accumFrames."""
        af = C.c_int32(0)
        check(lib().srt_checkpoint_load(self.ctx, str(path).encode(), C.byref(af)), "checkpoint_load")
        return int(af.value)

    def read_accum(self) -> np.ndarray:
        rows = self.local_rows()
        a = np.zeros((rows, self.width, 4), np.float32)
        check(lib().srt_read_accum(self.ctx, _ptr(a), a.nbytes), "read_accum")
        return a

    def write_accum(self, a: np.ndarray):
        a = np.ascontiguousarray(a, np.float32)
        check(lib().srt_write_accum(self.ctx, _ptr(a), a.nbytes), "write_accum")

    def read_output(self) -> np.ndarray:
        rows = self.local_rows()
        a = np.zeros((rows, self.width, 4), np.uint8)
        check(lib().srt_read_output(self.ctx, _ptr(a), a.nbytes), "read_output")
        return a

    def save_image(self, path: str | pathlib.Path, flip_y: bool = True) -> None:
        """image0 (the local rows) to a PNG / PPM file (write_image)."""
        check(lib().srt_write_output(self.ctx, str(path).encode(), int(flip_y)), "write_output")

    def trace_closest(self, rays: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """ray_intersects.glsl's closest-hit test kernel fed via UpdateRays (gpu_loader.cpp:198-210)."""
        rays = np.ascontiguousarray(rays, dtype=RAY_DTYPE)
        hits = np.zeros(len(rays), np.uint32)
        t = np.zeros(len(rays), np.float32)
        check(lib().srt_trace_closest(self.ctx, _ptr(rays), len(rays), _ptr(hits), _ptr(t)), "trace_closest")
        return hits, t


# ---------------------------------------------------------------------------
# AssetUtils upload API
# ---------------------------------------------------------------------------
def UploadModelDataToGPU(compute: Compute, models: Sequence[Model | None], binding_offset: int = 0) -> Scene:
    """AssetUtils::UploadModelDataToGPU (gpu_loader.cpp:63-183); raises RuntimeError('Model was null!')."""
    if any(m is None for m in models):
        raise RuntimeError("Model was null!")
    scene = Scene.from_models(models)
    compute.bind_scene(scene)
    return scene


def UpdateModelMatrix(compute: Compute, index: int, matrix) -> None:
    """AssetUtils::UpdateModelMatrix (gpu_loader.cpp:185-196); ``matrix`` is glm column-major (m[c][r])."""
    m = np.ascontiguousarray(np.asarray(matrix, np.float32).reshape(4, 4)).reshape(16)
    check(lib().srt_update_model_matrix(compute.ctx, index, _ptr(m)), "UpdateModelMatrix")
