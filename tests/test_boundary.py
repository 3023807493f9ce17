"""The drop-in boundary on the CPU: Compute::CreateComputeProgram's contract (srt_program_create) and the
reference's own upload path (gpu_loader.cpp:63-133, restated in tests/cpp/test_ref_loader.cpp) producing
exactly the std430 arrays srt_upload_scene takes.  No GPU call is made."""
import subprocess

import pytest

from conftest import OBJECTS, PKG, ROOT


def test_program_create_contract(tmp_path, capfd):
    """create_compute_program.h:46-72: a handle, or 0 with the log on stderr."""
    from srt_amd import _lib

    lib = _lib.lib()
    assert lib.srt_program_create(b"builtin:raytrace_compute") == _lib.SRT_PROGRAM_RAYTRACE
    assert lib.srt_program_create(b"builtin:ray_intersects") == _lib.SRT_PROGRAM_INTERSECT
    (tmp_path / "raytrace_compute.glsl").write_text("#version 450\n")
    (tmp_path / "ray_intersects.glsl").write_text("#version 450\n")
    (tmp_path / "blur.glsl").write_text("#version 450\n")
    assert lib.srt_program_create(str(tmp_path / "raytrace_compute.glsl").encode()) == _lib.SRT_PROGRAM_RAYTRACE
    assert lib.srt_program_create(str(tmp_path / "ray_intersects.glsl").encode()) == _lib.SRT_PROGRAM_INTERSECT
    assert lib.srt_program_create(str(tmp_path / "missing.glsl").encode()) == 0
    assert "err opening" in capfd.readouterr().err
    assert lib.srt_program_create(str(tmp_path / "blur.glsl").encode()) == 0
    assert "compile error" in capfd.readouterr().err
    assert lib.srt_program_create(None) == 0
    assert lib.srt_program_delete(_lib.SRT_PROGRAM_RAYTRACE) == _lib.SRT_OK
    assert lib.srt_program_delete(0) == _lib.SRT_ERR_INVALID


def test_python_compute_refuses_unknown_program(tmp_path):
    import srt_amd as S

    with pytest.raises(RuntimeError):
        S.Compute(str(tmp_path / "nope.glsl")).Init()


def _build(name):
    exe = ROOT / "tests" / "cpp" / "_build" / name
    exe.parent.mkdir(exist_ok=True)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", str(ROOT / "include"),
                    str(ROOT / "tests" / "cpp" / f"{name}.cpp"), "-o", str(exe), "-L", str(PKG), "-lsrt_amd",
                    f"-Wl,-rpath,{PKG}"], check=True)
    return exe


def test_reference_upload_path_builds_the_abi_arrays():
    """gpu_loader.cpp's flattening over two Models (with its index rebasing) yields, byte for byte, the
    arrays srt_upload_scene receives from srt_scene_build."""
    exe = _build("test_ref_loader")
    res = subprocess.run([str(exe), "arrays", str(OBJECTS) + "/"], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0 and res.stdout.startswith("OK arrays"), res.stdout + res.stderr


def test_model_host_arrays_shape():
    import ctypes as C

    import numpy as np
    import srt_amd as S
    from srt_amd import _lib

    m = S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")
    sizes = np.zeros(4, np.uint32)
    assert _lib.lib().srt_model_sizes(m.handle, C.c_void_p(sizes.ctypes.data)) == 0
    info = m.info()
    assert (sizes == [info["nodes"], info["triangles"], info["materials"], info["vertices"]]).all()
