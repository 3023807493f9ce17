"""Progressive renderer: the per-frame contract of src/main.cpp (:579-718) driven on the HIP kernels.

The reference app resets the accumulation buffer on the first frame
(EnableMouseCapture(false) sets the reset flag, input_handler.cpp:172), so frame
1 is a clear (accumFrames = 1) and frame k >= 2 traces sample index
k % (W*H).  After N sampled frames the displayed image is
sRGB(sum_{k=2}^{N+1} L_k / (N + 1)).
"""
from __future__ import annotations

import pathlib
from dataclasses import dataclass

import numpy as np

from . import (MODEL_LIGHTS, SPHERE_LIGHTS, Camera, Compute, Model, Scene, generate_noise, lights_array, load_obj,
               model_from_triangles)


@dataclass
class FrameSetup:
    """Everything the kernel reads, in reference layouts (also what the CPU oracle consumes)."""
    width: int
    height: int
    show_model: bool
    scene: Scene | None
    lights: np.ndarray
    noise: np.ndarray
    noise_u: np.ndarray
    camera: Camera
    max_depth: int = 5
    bvh_count: int = 1


def make_setup(width: int, height: int, *, show_model: bool, models=None, lights=None, max_depth: int = 5,
               bvh_count: int | None = None, gcc_order: bool = True, noise=None) -> FrameSetup:
    scene = Scene.from_models(models) if (show_model and models) else None
    if lights is None:
        lights = MODEL_LIGHTS if show_model else SPHERE_LIGHTS
    la = lights if isinstance(lights, np.ndarray) else lights_array(lights)
    if noise is None:
        noise = generate_noise(width, height, gcc_order)
    cam = Camera(show_model)
    if bvh_count is None:
        bvh_count = len(scene.bvhs) if scene is not None else 0
    return FrameSetup(width, height, show_model, scene, la, noise[0], noise[1], cam, max_depth, bvh_count)


class Renderer:
    """Drives one Compute context through the reference's progressive loop."""

    def __init__(self, setup: FrameSetup, *, device: int = 0, stream: int | None = None, rank: int = 0,
                 nranks: int = 1, band_rows: int = 16):
        self.setup = setup
        c = Compute("builtin:raytrace_compute", device=device, stream=stream).Init()
        self.compute = c
        c.Use()
        c.SetInt("Width", setup.width)
        c.SetInt("Height", setup.height)
        c.SetBool("showModel", setup.show_model)
        c.SetInt("maxDepth", setup.max_depth)
        c.SetUInt("bvh_count", setup.bvh_count)
        c.SetInt("lightCount", len(setup.lights))
        cam = setup.camera
        c.SetVec3("cameraOrigin", cam.getOrigin())
        c.SetVec3("cameraDirection", cam.getForward())
        c.SetVec3("cameraUp", cam.getUpVector())
        c.SetVec3("cameraRight", cam.getRightVector())
        c.bind_lights(setup.lights)
        c.bind_noise(setup.noise, setup.noise_u)
        if setup.scene is not None:
            c.bind_scene(setup.scene)
        c.set_tiling(rank, nranks, band_rows)
        c.alloc_images()
        self.accum_frames = 0

    @property
    def groups(self):
        s = self.setup
        return (s.width + 7) // 8, (s.height + 7) // 8

    def clear(self):
        """Frame 1 of the app: accumFrames = 1 with resetAccumBuffer = true."""
        self.accum_frames = 1
        c = self.compute
        c.SetBool("resetAccumBuffer", True)
        c.SetInt("accumFrames", self.accum_frames)
        c.Dispatch(*self.groups)
        c.SetBool("resetAccumBuffer", False)

    def frame(self):
        """One more progressive frame (one glDispatchCompute)."""
        self.accum_frames += 1
        c = self.compute
        c.SetBool("resetAccumBuffer", False)
        c.SetInt("accumFrames", self.accum_frames)
        c.Dispatch(*self.groups)

    def render(self, spp: int, *, count: bool = False, write_output: bool = True, clear: bool = True):
        """`spp` progressive frames in one fused launch (same accumulation as `spp` Dispatch calls)."""
        if clear:
            self.clear()
        first = self.accum_frames + 1
        self.compute.render_frames(first, spp, write_output=write_output, count=count)
        self.accum_frames += spp

    def finish(self):
        self.compute.Finish()

    def accum(self) -> np.ndarray:
        return self.compute.read_accum()

    def output(self) -> np.ndarray:
        return self.compute.read_output()

    def close(self):
        self.compute.close()


class GroupRenderer:
    """One frame tiled over several contexts of this process through the C ABI's device group
    (srt_group_*: row bands per context, one gather to context 0 -- RCCL across distinct devices, device
    copies when a device repeats -- and the full-frame assembly).  The same loop as Renderer."""

    def __init__(self, setup: FrameSetup, devices=(0,), *, band_rows: int = 8):
        import ctypes as C

        from ._lib import check, lib

        self.setup = setup
        self.parts = [Renderer(setup, device=d) for d in devices]
        ctxs = (C.c_void_p * len(devices))(*[r.compute.ctx for r in self.parts])
        g = C.c_void_p()
        check(lib().srt_group_create(ctxs, len(devices), band_rows, C.byref(g)), "group_create")
        self.g = g
        check(lib().srt_group_alloc_images(g), "group_alloc_images")
        self.accum_frames = 0

    @property
    def transport(self) -> str:
        from ._lib import lib

        return lib().srt_group_transport(self.g).decode()

    def get_int(self, name: str) -> int:
        """srt_group_get_int: "contexts", "ranks" (RCCL's communicator count), "gathers.output",
        "gathers.accum", "bytes.output" / "bytes.accum" (KiB one such gather moves)."""
        import ctypes as C

        from ._lib import check, lib

        v = C.c_int()
        check(lib().srt_group_get_int(self.g, name.encode(), C.byref(v)), "group_get_int")
        return int(v.value)

    def kernel_ms(self) -> list[float]:
        """Each context's sample-kernel device time in the last render (HIP events on its stream)."""
        import ctypes as C

        from ._lib import check, lib

        ms = (C.c_float * len(self.parts))()
        check(lib().srt_group_last_kernel_ms(self.g, ms, len(self.parts)), "group_last_kernel_ms")
        return [float(x) for x in ms]

    def kernel_time(self) -> list[tuple[float, int]]:
        """Each context's (sample-kernel throughput ms, launches) since the previous call
        (srt_group_kernel_time): a timed loop of group renders enqueued back to back reads it once."""
        import ctypes as C

        from ._lib import check, lib

        n = len(self.parts)
        ms, k = (C.c_double * n)(), (C.c_int * n)()
        check(lib().srt_group_kernel_time(self.g, ms, k, n), "group_kernel_time")
        return [(float(ms[i]), int(k[i])) for i in range(n)]

    def exchange_time(self) -> list[tuple[float, int]]:
        """Each context's (ms in its part of the per-frame sRGB8 exchange, frames) since the previous call
        (srt_group_exchange_time; context 0's part includes the assembly)."""
        import ctypes as C

        from ._lib import check, lib

        n = len(self.parts)
        ms, k = (C.c_double * n)(), (C.c_int * n)()
        check(lib().srt_group_exchange_time(self.g, ms, k, n), "group_exchange_time")
        return [(float(ms[i]), int(k[i])) for i in range(n)]

    def count(self, spp: int) -> dict:
        """Untimed counting render (the counting instance on every context, CheckHit counts summed) of
        the reset frame + `spp` frames.  The contexts' radiance is left at the rendered frame; the group's
        image0 is not assembled (the timed renders that follow do that)."""
        self.finish()
        self.clear()
        for p in self.parts:
            p.compute.render_frames(2, spp, write_output=True, count=True)
        self.accum_frames = spp + 1
        self.finish()
        tot: dict = {}
        self.part_stats = [p.compute.stats() for p in self.parts]  # each context's share of the counts
        for st in self.part_stats:
            for k, v in st.items():
                tot[k] = max(tot.get(k, 0), v) if k == "max_stack" else tot.get(k, 0) + v
        return tot

    @property
    def groups(self):
        s = self.setup
        return (s.width + 7) // 8, (s.height + 7) // 8

    def _set(self, reset: bool):
        from ._lib import check, lib

        check(lib().srt_group_set_bool(self.g, b"resetAccumBuffer", int(reset)), "group_set_bool")
        check(lib().srt_group_set_int(self.g, b"accumFrames", self.accum_frames), "group_set_int")

    def clear(self):
        from ._lib import check, lib

        self.accum_frames = 1
        self._set(True)
        check(lib().srt_group_dispatch(self.g, *self.groups), "group_dispatch")
        self._set(False)

    def frame(self):
        from ._lib import check, lib

        self.accum_frames += 1
        self._set(False)
        check(lib().srt_group_dispatch(self.g, *self.groups), "group_dispatch")

    def render(self, spp: int, *, clear: bool = True):
        from ._lib import check, lib

        if clear:
            self.clear()
        check(lib().srt_group_render_frames(self.g, self.accum_frames + 1, spp), "group_render_frames")
        self.accum_frames += spp

    def finish(self):
        from ._lib import check, lib

        check(lib().srt_group_finish(self.g), "group_finish")

    def accum(self) -> np.ndarray:
        from ._lib import check, lib

        s = self.setup
        a = np.zeros((s.height, s.width, 4), np.float32)
        check(lib().srt_group_read_accum(self.g, a.ctypes.data, a.nbytes), "group_read_accum")
        return a

    def output(self) -> np.ndarray:
        from ._lib import check, lib

        s = self.setup
        o = np.zeros((s.height, s.width, 4), np.uint8)
        check(lib().srt_group_read_output(self.g, o.ctypes.data, o.nbytes), "group_read_output")
        return o

    def close(self):
        from ._lib import lib

        if self.g is not None:
            lib().srt_group_destroy(self.g)
            self.g = None
        for r in self.parts:
            r.close()


def rubik_model(objects_dir: str | pathlib.Path) -> Model:
    return load_obj(pathlib.Path(objects_dir) / "Rubik" / "Rubik.obj")


def splitmix64_uniform(n: int, seed: int = 0x5EED2025) -> np.ndarray:
    """n uniforms in [0, 1) as float32: SplitMix64 stream, top 24 bits * 2^-24."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)
    idx = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)) & M
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return ((z >> np.uint64(40)).astype(np.float32)) * np.float32(2.0 ** -24)


def synthetic_triangles(n_tris: int, seed: int = 0x5EED2025) -> np.ndarray:
    """centres U([-10,10]x[0,18]x[-10,10]), vertices = centre + U(-0.05,0.05)^3."""
    u = splitmix64_uniform(12 * n_tris, seed).reshape(n_tris, 12)
    lo = np.array([-10.0, 0.0, -10.0], np.float32)
    ext = np.array([20.0, 18.0, 20.0], np.float32)
    c = lo + ext * u[:, 0:3]
    tri = np.empty((n_tris, 3, 3), np.float32)
    for k in range(3):
        tri[:, k, :] = c + (np.float32(-0.05) + np.float32(0.1) * u[:, 3 + 3 * k:6 + 3 * k])
    return tri.reshape(n_tris, 9)


def torus_knot_grid(n_u: int = 512, n_v: int = 256, p: int = 2, q: int = 3, scale: float = 1.0) -> np.ndarray:
    """The (n_u, n_v, 3) float64 vertex grid of torus_knot_triangles' tube (u along the knot, v around it),
    `scale` times the unit size about the centre (0, 9, 0)."""
    u = np.arange(n_u, dtype=np.float64) * (2.0 * np.pi / n_u)
    v = np.arange(n_v, dtype=np.float64) * (2.0 * np.pi / n_v)

    def curve(t):
        r = 6.0 + 2.6 * np.cos(q * t)
        return np.stack([r * np.cos(p * t), 9.0 + r * np.sin(p * t), 4.0 * np.sin(q * t)], axis=-1)

    c = curve(u)
    tang = curve(u + 1e-4) - curve(u - 1e-4)
    tang /= np.linalg.norm(tang, axis=-1, keepdims=True)
    up = np.array([0.0, 0.0, 1.0])
    n1 = np.cross(tang, up)
    n1 /= np.linalg.norm(n1, axis=-1, keepdims=True)
    n2 = np.cross(tang, n1)
    rad = 2.4
    g = c[:, None, :] + rad * (np.cos(v)[None, :, None] * n1[:, None, :] + np.sin(v)[None, :, None] * n2[:, None, :])
    if scale != 1.0:
        ctr = np.array([0.0, 9.0, 0.0])
        g = ctr + scale * (g - ctr)
    return g


# The surface-mesh stand-in's size: the unit knot covers 22% of the model camera's frame, so 81% of its rays
# would be camera and shadow rays; at 1.5 it fills about half of it, as a framed model does, and 29% of the
# counted rays are bounce rays (oracle, 192x108 @ 4 spp).  The Airplane-material knot keeps the unit size.
SURFACE_KNOT_SCALE = 1.5


def torus_knot_triangles(n_u: int = 512, n_v: int = 256, p: int = 2, q: int = 3, outward: bool = True,
                         scale: float = 1.0) -> np.ndarray:
    """A closed surface mesh for the global-scene path (the Airplane OBJ is absent): a (p, q) torus-knot tube,
    2 * n_u * n_v triangles, centred at (0, 9, 0) in the Rubik's extent (~18 units across) so the model camera
    and lights of src/main.cpp frame it.  Deterministic (float64 numpy, rounded once to float32).

    `outward` (the default): faces wound so that the geometric normal normalize(cross(e1, e2)), which the shader
    uses as is (ray_intersects.glsl:90, raytrace_compute.glsl:157: not face-forwarded), points out of the tube,
    as an exported model's does, so paths bounce off it.  `outward=False` is the inward winding of rounds 2-5
    (first_hit_only_knot_model): SampleIndirectNew rejects every bounce there (dot(N, V) <= 0, brdf.glsl:242),
    so a path ends after its first hit's shadow ray."""
    pts = torus_knot_grid(n_u, n_v, p, q, scale)
    i0 = np.arange(n_u)[:, None]
    j0 = np.arange(n_v)[None, :]
    i1, j1 = (i0 + 1) % n_u, (j0 + 1) % n_v
    a, b, cc, d = pts[i0, j0], pts[i1, j0], pts[i1, j1], pts[i0, j1]
    if outward:
        tri = np.stack([np.stack([a, cc, b], axis=-2), np.stack([a, d, cc], axis=-2)], axis=2)
    else:
        tri = np.stack([np.stack([a, b, cc], axis=-2), np.stack([a, cc, d], axis=-2)], axis=2)  # (n_u, n_v, 2, 3, 3)
    return tri.reshape(-1, 9).astype(np.float32)


def write_textured_torus_knot_obj(path: str | pathlib.Path, mtllib: str, materials, n_u: int = 512, n_v: int = 256,
                                  s_repeat: float = 3.0, outward: bool = True) -> pathlib.Path:
    """The torus-knot tube as an OBJ with texture coordinates and several materials: `materials` (usemtl
    names of the .mtl `mtllib`, which lies next to `path` with its textures) take equal consecutive
    segments along the knot, and vertex (i, j) of the grid carries vt (s_repeat * i / n_u, j / n_v) --
    the texture repeats s_repeat times along the knot (GL_REPEAT) and once around the tube.  Loaded with
    SRT_LOAD_TEXCOORDS (the loader with has_texcoords set) every hit samples its material's texture at its
    interpolated uv.  Positions are the float32 grid written with 9 significant digits (exact round trip).
    `outward`: faces wound so that the geometric normal (normalize(cross(e1, e2)), which the shader uses as
    is, ray_intersects.glsl:95) points out of the tube, as an exported model's does -- paths then bounce off
    the surface (SampleIndirectNew rejects dot(N, V) <= 0, brdf.glsl:239-277); torus_knot_triangles' winding
    points inward, so its paths end at the first hit after the shadow ray."""
    path = pathlib.Path(path)
    pts = torus_knot_grid(n_u, n_v).astype(np.float32).reshape(-1, 3)
    i, j = np.meshgrid(np.arange(n_u), np.arange(n_v), indexing="ij")
    st = np.stack([np.float32(s_repeat) * i.astype(np.float32) / np.float32(n_u),
                   j.astype(np.float32) / np.float32(n_v)], axis=-1).reshape(-1, 2)
    lines = [f"mtllib {mtllib}"]
    lines += [f"v {x:.9g} {y:.9g} {z:.9g}" for x, y, z in pts.tolist()]
    lines += [f"vt {a:.9g} {b:.9g}" for a, b in st.tolist()]
    idx = lambda a, b: (a % n_u) * n_v + (b % n_v) + 1  # noqa: E731  (1-based, vertex and vt alike)
    nm = len(materials)
    for seg, m in enumerate(materials):
        lines.append(f"usemtl {m}")
        for a in range(seg * n_u // nm, (seg + 1) * n_u // nm):
            for b in range(n_v):
                A, B, C, D = idx(a, b), idx(a + 1, b), idx(a + 1, b + 1), idx(a, b + 1)
                if outward:
                    lines.append(f"f {A}/{A} {C}/{C} {B}/{B}")
                    lines.append(f"f {A}/{A} {D}/{D} {C}/{C}")
                else:
                    lines.append(f"f {A}/{A} {B}/{B} {C}/{C}")
                    lines.append(f"f {A}/{A} {C}/{C} {D}/{D}")
    path.write_text("\n".join(lines) + "\n")
    return path


def torus_knot_model(n_u: int = 512, n_v: int = 256, outward: bool = True,
                     scale: float = SURFACE_KNOT_SCALE) -> Model:
    """The surface-mesh stand-in for C3's regime (bench.py's surface_mesh leg): the outward-wound knot at
    SURFACE_KNOT_SCALE, paths bouncing off it."""
    return model_from_triangles(torus_knot_triangles(n_u, n_v, outward=outward, scale=scale), kd=(0.8, 0.6, 0.3),
                                ks=(0.5, 0.5, 0.5), ns=40.0)


def first_hit_only_knot_model(n_u: int = 512, n_v: int = 256) -> Model:
    """The surface-mesh leg of rounds 2-5: the unit-size knot wound inward, so no path bounces
    (torus_knot_triangles(outward=False)); kept for comparisons only."""
    return torus_knot_model(n_u, n_v, outward=False, scale=1.0)


def synthetic_model(n_tris: int, seed: int = 0x5EED2025) -> Model:
    return model_from_triangles(synthetic_triangles(n_tris, seed), kd=(0.8, 0.8, 0.8), ks=(0.0, 0.0, 0.0), ns=10.0)
