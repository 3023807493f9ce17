"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It consumes the reference std430 arrays (numpy structured
arrays with the dtypes of srt_amd) and reproduces raytrace_compute.glsl's
dispatches on the CPU (see srt_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib
import subprocess

import numpy as np

ORACLE_DIR = pathlib.Path(__file__).resolve().parent


def _host_has_fma() -> bool:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                return " fma " in f" {line.split(':', 1)[1].strip()} "
    except OSError:
        pass
    return False


# liboracle.so is built with -mfma (hardware fmaf, the same bits as libm's); a CPU without FMA loads
# the generic build of the same source
LIB = pathlib.Path(os.environ.get("ORACLE_LIB_PATH", ORACLE_DIR / "_build" / (
    "liboracle.so" if _host_has_fma() else "liboracle_generic.so")))
# contract variants of the tolerance measurement (srt_oracle.c ORACLE_CONTRACT): "A" is the kernel's
CONTRACTS = ("A", "B", "C", "D", "E")

P = C.c_void_p


class OrScene(C.Structure):
    _fields_ = [("bvhs", P), ("n_bvhs", C.c_uint32), ("nodes", P), ("n_nodes", C.c_uint32), ("mats", P),
                ("n_mats", C.c_uint32), ("tex_albedo", P), ("tris", P), ("n_tris", C.c_uint32), ("verts", P),
                ("n_verts", C.c_uint32), ("lights", P), ("n_lights", C.c_uint32), ("noise", P), ("noise_u", P),
                ("tex_texels", P), ("tex_info", P), ("n_tex", C.c_uint32)]


class OrFrame(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("accum_frames", C.c_int), ("reset", C.c_int),
                ("show_model", C.c_int), ("bvh_count", C.c_uint32), ("light_count", C.c_int),
                ("max_depth", C.c_int), ("cam_origin", C.c_float * 3), ("cam_dir", C.c_float * 3),
                ("cam_up", C.c_float * 3), ("cam_right", C.c_float * 3)]


class OrStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("rays", "nodes", "tris", "rng_u", "rng_sq", "light_reads",
                                           "mat_reads", "samples", "stack_overflow", "max_stack",
                                           "shadow_rays")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


_libs: dict = {}


def build():
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def lib(contract: str = "A"):
    """The oracle library of contract variant `contract` (A: the kernel's contract)."""
    if contract not in _libs:
        path = LIB if contract == "A" else ORACLE_DIR / "_build" / f"liboracle_{contract}.so"
        if not path.exists():
            build()
        L = C.CDLL(str(path))
        L.oracle_dispatch.argtypes = [C.POINTER(OrScene), C.POINTER(OrFrame), P, P, C.c_int, C.c_int,
                                      C.POINTER(OrStats)]
        L.oracle_render.argtypes = [C.POINTER(OrScene), C.POINTER(OrFrame), C.c_int, C.c_int, P, P, C.c_int,
                                    C.c_int, C.c_int, C.POINTER(OrStats)]
        L.oracle_render_rows.argtypes = [C.POINTER(OrScene), C.POINTER(OrFrame), C.c_int, C.c_int, P, P, P, C.c_int,
                                         C.c_int, C.POINTER(OrStats)]
        L.oracle_trace_closest.argtypes = [C.POINTER(OrScene), C.c_uint32, P, C.c_int, P, P, P, C.POINTER(OrStats)]
        for fn in ("oracle_sin", "oracle_cos"):
            getattr(L, fn).argtypes = [C.c_float]
            getattr(L, fn).restype = C.c_float
        L.oracle_pow.argtypes = [C.c_float, C.c_float]
        L.oracle_pow.restype = C.c_float
        L.oracle_pow5.argtypes = [C.c_float]
        L.oracle_pow5.restype = C.c_float
        L.oracle_rand_float.argtypes = [C.c_float, C.c_float]
        L.oracle_rand_float.restype = C.c_float
        L.oracle_contract.restype = C.c_int
        if chr(L.oracle_contract()) != contract:
            raise RuntimeError(f"{path}: built for contract {chr(L.oracle_contract())}, not {contract}")
        _libs[contract] = L
    return _libs[contract]


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


class Oracle:
    """Holds the reference-layout inputs of one scene + noise + lights."""

    def __init__(self, scene=None, lights=None, noise=None, noise_u=None, contract: str = "A"):
        self._lib = lib(contract)
        self._keep = []
        s = OrScene()
        if scene is not None:
            arrs = [np.ascontiguousarray(getattr(scene, k)) for k in ("bvhs", "nodes", "mats", "tex_albedo", "tris",
                                                                      "verts")]
            self._keep += arrs
            bvhs, nodes, mats, tex, tris, verts = arrs
            s.bvhs, s.n_bvhs = _p(bvhs), len(bvhs)
            s.nodes, s.n_nodes = _p(nodes), len(nodes)
            s.mats, s.n_mats = _p(mats), len(mats)
            s.tris, s.n_tris = _p(tris), len(tris)
            s.verts, s.n_verts = _p(verts), len(verts)
            if getattr(scene, "sample_textures", False):
                # TriangleToSupportedMat samples texture `handle` at the hit's uv
                texs = [t if t.ndim == 3 else t[:, :, None] for t in scene.textures]
                info = np.zeros((max(len(texs), 1), 4), np.uint32)
                first = 0
                for i, t in enumerate(texs):
                    info[i] = (first, t.shape[1], t.shape[0], t.shape[2])
                    first += t.shape[0] * t.shape[1] * t.shape[2]
                texels = np.concatenate([t.reshape(-1) for t in texs] or [np.zeros(1, np.uint8)]).astype(np.uint8)
                self._keep += [info, texels]
                s.tex_texels, s.tex_info, s.n_tex = _p(texels), _p(info), len(texs)
            else:
                s.tex_albedo = _p(np.ascontiguousarray(tex, np.float32))
        if lights is not None:
            la = np.ascontiguousarray(lights)
            self._keep.append(la)
            s.lights, s.n_lights = _p(la), len(la)
        if noise is not None:
            n = np.ascontiguousarray(noise, np.float32)
            nu = np.ascontiguousarray(noise_u, np.float32)
            self._keep += [n, nu]
            s.noise, s.noise_u = _p(n), _p(nu)
        self.scene = s

    @staticmethod
    def frame(width, height, *, accum_frames=1, reset=False, show_model=True, bvh_count=1, light_count=0,
              max_depth=5, origin=(0, 0, 0), direction=(0, 0, -1), up=(0, 1, 0), right=(1, 0, 0)) -> OrFrame:
        f = OrFrame()
        f.width, f.height, f.accum_frames, f.reset = width, height, accum_frames, int(reset)
        f.show_model, f.bvh_count, f.light_count, f.max_depth = int(show_model), bvh_count, light_count, max_depth
        for name, v in (("cam_origin", origin), ("cam_dir", direction), ("cam_up", up), ("cam_right", right)):
            arr = getattr(f, name)
            for i in range(3):
                arr[i] = float(np.float32(v[i]))
        return f

    def dispatch(self, f: OrFrame, accum: np.ndarray, out: np.ndarray, y0=0, y1=None) -> dict:
        st = OrStats()
        self._lib.oracle_dispatch(C.byref(self.scene), C.byref(f), _p(accum), _p(out), y0,
                              f.height if y1 is None else y1, C.byref(st))
        return st.as_dict()

    def render(self, f: OrFrame, frame_first: int, nframes: int, accum: np.ndarray, out: np.ndarray, y0=0, y1=None,
               threads=0) -> dict:
        st = OrStats()
        self._lib.oracle_render(C.byref(self.scene), C.byref(f), frame_first, nframes, _p(accum), _p(out), y0,
                            f.height if y1 is None else y1, threads, C.byref(st))
        return st.as_dict()

    def render_rows(self, f: OrFrame, frame_first: int, nframes: int, accum: np.ndarray, out: np.ndarray, rows,
                    threads=0) -> dict:
        rows = np.ascontiguousarray(rows, np.int32)
        st = OrStats()
        self._lib.oracle_render_rows(C.byref(self.scene), C.byref(f), frame_first, nframes, _p(accum), _p(out), _p(rows),
                                 len(rows), threads, C.byref(st))
        return st.as_dict()

    def trace_closest(self, bvh_count: int, rays: np.ndarray):
        rays = np.ascontiguousarray(rays)
        n = len(rays)
        hits = np.zeros(n, np.uint32)
        t = np.zeros(n, np.float32)
        nrm = np.zeros((n, 3), np.float32)
        st = OrStats()
        self._lib.oracle_trace_closest(C.byref(self.scene), bvh_count, _p(rays), n, _p(hits), _p(t), _p(nrm),
                                   C.byref(st))
        return hits, t, nrm, st.as_dict()


def sin(x):
    return lib().oracle_sin(float(x))


def cos(x):
    return lib().oracle_cos(float(x))


def pow(x, y):  # noqa: A001
    return lib().oracle_pow(float(x), float(y))


def pow5(x):
    return lib().oracle_pow5(float(x))


def rand_float(sx, sy):
    return lib().oracle_rand_float(float(sx), float(sy))
