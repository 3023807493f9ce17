"""Test configuration: paths, the `gpu` marker, shared helpers.

CPU tests (-m "not gpu") pin the oracle against the reference's known answers,
check the host producers against an independent restatement, check the C ABI
library loads and exports its header, and run the multi-rank logic on gloo.
GPU tests (-m gpu) are the parity tests proper: HIP kernels vs the oracle.
"""
from __future__ import annotations

import os
import pathlib
import subprocess
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
PKG = ROOT / "simple-ray-tracer_amd"
GOLDEN = ROOT / "tests" / "golden"
OBJECTS = GOLDEN / "objects"
for p in (str(PKG), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels); run with -m gpu")


def _ensure_built():
    if not (PKG / "libsrt_amd.so").exists():
        subprocess.run(["make", "-s", "-C", str(PKG)], check=True)
    if not (ROOT / "oracle" / "_build" / "liboracle.so").exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def rubik_path():
    return OBJECTS / "Rubik" / "Rubik.obj"


def bits_equal(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Bitwise equality of float arrays, any NaN equal to any NaN (NaN payloads are not specified
    by IEEE 754 and differ between x86 and gfx950)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    same = a.view(np.uint32) == b.view(np.uint32)
    return same | (np.isnan(a) & np.isnan(b))


def oracle_render(setup, spp: int, rows=None, threads: int = 0, contract: str = "A"):
    """Reset frame + `spp` progressive frames on the CPU oracle (full frame or given rows), in the
    kernel's arithmetic contract or one of the variants (oracle/srt_oracle.c ORACLE_CONTRACT)."""
    from oracle import pyoracle as O

    s = setup
    orc = O.Oracle(s.scene, s.lights, s.noise, s.noise_u, contract=contract)
    cam = s.camera
    f = O.Oracle.frame(s.width, s.height, show_model=s.show_model, bvh_count=s.bvh_count, light_count=len(s.lights),
                       max_depth=s.max_depth, origin=cam.position, direction=cam.front, up=cam.up, right=cam.right)
    acc = np.zeros((s.height, s.width, 4), np.float32)
    out = np.zeros((s.height, s.width, 4), np.uint8)
    f.reset, f.accum_frames = 1, 1
    orc.dispatch(f, acc, out)
    f.reset = 0
    if rows is None:
        st = orc.render(f, 2, spp, acc, out, threads=threads)
    else:
        st = orc.render_rows(f, 2, spp, acc, out, rows, threads=threads)
    return acc, out, st
