"""ctypes binding of libsrt_amd.so (include/srt_amd.h).

The shared library is built in-tree (``make -C simple-ray-tracer_amd``) and is
the only compute path: there is no CPU or PyTorch fallback.  Loading fails
loudly when the library is missing.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

PKG_DIR = pathlib.Path(__file__).resolve().parent.parent
LIB_PATH = pathlib.Path(os.environ.get("SRT_LIB_PATH", PKG_DIR / "libsrt_amd.so"))

SRT_OK = 0
SRT_ERR_INVALID = 1
SRT_ERR_HIP = 2
SRT_ERR_NOT_FOUND = 3
SRT_ERR_IO = 4
SRT_ERR_STATE = 5
SRT_ERR_LIMIT = 6
SRT_PROGRAM_RAYTRACE = 1
SRT_PROGRAM_INTERSECT = 2


class BvhRecord(C.Structure):
    _fields_ = [("first_index", C.c_uint32), ("count", C.c_uint32), ("pad0", C.c_uint32),
                ("pad1", C.c_uint32), ("frame", C.c_float * 16)]


class BvhNode(C.Structure):
    _fields_ = [("min_bounds", C.c_float * 3), ("first_child_or_prim_index", C.c_uint32),
                ("max_bounds", C.c_float * 3), ("prim_count", C.c_uint32)]


class MaterialObj(C.Structure):
    _fields_ = [("diffuse", C.c_float * 3), ("specular_ex", C.c_float), ("specular", C.c_float * 3),
                ("use_texture", C.c_uint32), ("handle", C.c_uint32 * 2), ("pad0", C.c_uint32),
                ("pad1", C.c_uint32)]


class Triangle(C.Structure):
    _fields_ = [("v0_idx", C.c_uint32), ("v1_idx", C.c_uint32), ("v2_idx", C.c_uint32),
                ("material_idx", C.c_uint32)]


class Vertex(C.Structure):
    _fields_ = [("vertex", C.c_float * 3), ("pad0", C.c_float), ("texture", C.c_float * 2),
                ("pad1", C.c_float * 2)]


class Light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("intensity", C.c_float), ("color", C.c_float * 3),
                ("pad1", C.c_float)]


class CameraState(C.Structure):
    """srt_camera: RayTracer::Camera's interactive state (include/raytracer/camera.h:30-96)."""
    _fields_ = [("position", C.c_float * 3), ("front", C.c_float * 3), ("up", C.c_float * 3),
                ("right", C.c_float * 3), ("yaw", C.c_float), ("pitch", C.c_float), ("show_model", C.c_int32),
                ("frame_counter", C.c_int32)]


class Ray(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("pad0", C.c_float), ("direction", C.c_float * 3),
                ("intersection_distance", C.c_float)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("rays", "nodes", "tris", "rng_u", "rng_sq", "light_reads",
                                           "mat_reads", "samples", "stack_overflow", "max_stack", "bounce_cap")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class Texture(C.Structure):
    _fields_ = [("texels", C.c_void_p), ("width", C.c_int32), ("height", C.c_int32), ("channels", C.c_int32)]


assert C.sizeof(BvhRecord) == 80 and C.sizeof(BvhNode) == 32 and C.sizeof(MaterialObj) == 48
assert C.sizeof(Triangle) == 16 and C.sizeof(Vertex) == 32 and C.sizeof(Light) == 32 and C.sizeof(Ray) == 32

P = C.c_void_p
_SIGS = {
    "srt_last_error": (C.c_char_p, []),
    "srt_abi_version": (C.c_int, []),
    "srt_code_hash": (C.c_char_p, []),
    "srt_create": (C.c_int, [C.c_int, P, C.POINTER(P)]),
    "srt_program_create": (C.c_uint32, [C.c_char_p]),
    "srt_program_delete": (C.c_int, [C.c_uint32]),
    "srt_destroy": (C.c_int, [P]),
    "srt_stream": (P, [P]),
    "srt_set_bool": (C.c_int, [P, C.c_char_p, C.c_int]),
    "srt_set_int": (C.c_int, [P, C.c_char_p, C.c_int]),
    "srt_set_uint": (C.c_int, [P, C.c_char_p, C.c_uint32]),
    "srt_set_float": (C.c_int, [P, C.c_char_p, C.c_float]),
    "srt_set_vec3": (C.c_int, [P, C.c_char_p, C.c_float, C.c_float, C.c_float]),
    "srt_dispatch": (C.c_int, [P, C.c_uint32, C.c_uint32]),
    "srt_finish": (C.c_int, [P]),
    "srt_render_frames": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int]),
    "srt_get_stats": (C.c_int, [P, C.POINTER(Stats)]),
    "srt_ray_kinds": (C.c_int, [P, P]),
    "srt_last_kernel_ms": (C.c_int, [P, C.POINTER(C.c_float)]),
    "srt_kernel_time": (C.c_int, [P, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "srt_reset_stats": (C.c_int, [P]),
    "srt_nan_samples": (C.c_int, [P, C.POINTER(C.c_uint64)]),
    "srt_checkpoint_save": (C.c_int, [P, C.c_char_p]),
    "srt_checkpoint_load": (C.c_int, [P, C.c_char_p, C.POINTER(C.c_int32)]),
    "srt_set_tiling": (C.c_int, [P, C.c_int, C.c_int, C.c_int]),
    "srt_local_rows": (C.c_int, [P]),
    "srt_device": (C.c_int, [P]),
    "srt_get_int": (C.c_int, [P, C.c_char_p, C.POINTER(C.c_int)]),
    "srt_group_create": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, C.POINTER(P)]),
    "srt_group_destroy": (C.c_int, [P]),
    "srt_group_set_bool": (C.c_int, [P, C.c_char_p, C.c_int]),
    "srt_group_set_int": (C.c_int, [P, C.c_char_p, C.c_int]),
    "srt_group_set_uint": (C.c_int, [P, C.c_char_p, C.c_uint32]),
    "srt_group_set_vec3": (C.c_int, [P, C.c_char_p, C.c_float, C.c_float, C.c_float]),
    "srt_group_alloc_images": (C.c_int, [P]),
    "srt_group_dispatch": (C.c_int, [P, C.c_uint32, C.c_uint32]),
    "srt_group_render_frames": (C.c_int, [P, C.c_int, C.c_int]),
    "srt_group_finish": (C.c_int, [P]),
    "srt_group_read_accum": (C.c_int, [P, P, C.c_size_t]),
    "srt_group_read_output": (C.c_int, [P, P, C.c_size_t]),
    "srt_group_image_pointers": (C.c_int, [P, C.POINTER(P), C.POINTER(P)]),
    "srt_group_transport": (C.c_char_p, [P]),
    "srt_group_get_int": (C.c_int, [P, C.c_char_p, C.POINTER(C.c_int)]),
    "srt_group_last_kernel_ms": (C.c_int, [P, C.POINTER(C.c_float), C.c_int]),
    "srt_group_kernel_time": (C.c_int, [P, C.POINTER(C.c_double), C.POINTER(C.c_int), C.c_int]),
    "srt_group_exchange_time": (C.c_int, [P, C.POINTER(C.c_double), C.POINTER(C.c_int), C.c_int]),
    "srt_upload_scene": (C.c_int, [P, P, C.c_uint32, P, C.c_uint32, P, P, C.c_uint32, P, C.c_uint32, P,
                                   C.c_uint32]),
    "srt_upload_textures": (C.c_int, [P, C.POINTER(Texture), C.c_uint32]),
    "srt_texture_sample": (C.c_int, [C.POINTER(Texture), C.c_float, C.c_float, P]),
    "srt_update_model_matrix": (C.c_int, [P, C.c_uint32, P]),
    "srt_set_lights": (C.c_int, [P, P, C.c_uint32]),
    "srt_set_noise": (C.c_int, [P, P, P, C.c_size_t]),
    "srt_alloc_images": (C.c_int, [P]),
    "srt_read_accum": (C.c_int, [P, P, C.c_size_t]),
    "srt_read_output": (C.c_int, [P, P, C.c_size_t]),
    "srt_image_write": (C.c_int, [C.c_char_p, P, C.c_int, C.c_int, C.c_int]),
    "srt_write_output": (C.c_int, [P, C.c_char_p, C.c_int]),
    "srt_write_accum": (C.c_int, [P, P, C.c_size_t]),
    "srt_image_pointers": (C.c_int, [P, C.POINTER(P), C.POINTER(P)]),
    "srt_set_image_buffers": (C.c_int, [P, P, P]),
    "srt_assemble_bands": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "srt_assemble_output_bands": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, P]),
    "srt_trace_closest": (C.c_int, [P, P, C.c_uint32, P, P]),
    "srt_model_load": (C.c_int, [C.c_char_p, C.POINTER(P)]),
    "srt_model_load_ex": (C.c_int, [C.c_char_p, C.c_uint32, C.POINTER(P)]),
    "srt_model_from_triangles": (C.c_int, [P, C.c_uint32, P, P, C.c_float, C.POINTER(P)]),
    "srt_model_free": (C.c_int, [P]),
    "srt_model_info": (C.c_int, [P, P, P, P]),
    "srt_model_sizes": (C.c_int, [P, P]),
    "srt_model_copy": (C.c_int, [P, P, P, P, P]),
    "srt_model_prim_order": (C.c_int, [P, P]),
    "srt_scene_build": (C.c_int, [P, C.c_uint32, C.POINTER(P)]),
    "srt_scene_free": (C.c_int, [P]),
    "srt_scene_sizes": (C.c_int, [P, P]),
    "srt_scene_copy": (C.c_int, [P, P, P, P, P, P, P]),
    "srt_scene_tri_order": (C.c_int, [P, P]),
    "srt_scene_texture_count": (C.c_int, [P, C.POINTER(C.c_uint32), C.POINTER(C.c_int)]),
    "srt_scene_texture": (C.c_int, [P, C.c_uint32, C.POINTER(Texture)]),
    "srt_upload_scene_obj": (C.c_int, [P, P]),
    "srt_noise_generate": (C.c_int, [C.c_uint32, C.c_int, P, P]),
    "srt_glibc_rand": (C.c_int, [C.c_uint32, P]),
    "srt_camera_reset": (C.c_int, [C.c_int, P, P, P, P]),
    "srt_camera_basis": (C.c_int, [C.c_float, C.c_float, P, P, P]),
    "srt_camera_init": (C.c_int, [C.POINTER(CameraState), C.c_int]),
    "srt_camera_state_reset": (C.c_int, [C.POINTER(CameraState)]),
    "srt_camera_move": (C.c_int, [C.POINTER(CameraState), C.c_int, C.c_float]),
    "srt_camera_rotate": (C.c_int, [C.POINTER(CameraState), C.c_float, C.c_float]),
    "srt_camera_move_and_rotate": (C.c_int, [C.POINTER(CameraState), C.c_float, P, P, C.c_float]),
    "srt_progressive_frame": (C.c_int, [C.POINTER(CameraState), P, P, C.c_int, C.POINTER(C.c_int32), C.c_float,
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


class SrtError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed with status {code}: {last_error()}")
        self.code = code


def lib() -> C.CDLL:
    """Load libsrt_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(f"{LIB_PATH} not built: run `make -C {PKG_DIR}` (or __graft_entry__.build())")
        # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7 / libhsa-runtime64.so.1
        # (same sonames as /opt/rocm's), so whichever is loaded first serves both.  Loading ours
        # first and torch's CUDA later left torch on a runtime it was not built against, and the
        # process aborted at exit ("free(): invalid pointer") after a test had used torch.cuda
        # buffers; with torch loaded first, as bench.py does, both run on torch's runtime.
        # A pure C-ABI user that never touches torch may skip it: SRT_PRELOAD_TORCH=0.
        if os.environ.get("SRT_PRELOAD_TORCH", "1") != "0":
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        handle = C.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def last_error() -> str:
    if _lib is None:
        return ""
    msg = _lib.srt_last_error()
    return msg.decode() if msg else ""


def check(code: int, what: str) -> int:
    if code != SRT_OK:
        raise SrtError(code, what)
    return code
