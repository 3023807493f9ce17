"""The C-ABI library loads and exports every entry point include/srt_amd.h declares (CPU only)."""
import ctypes
import re
import subprocess

import pytest

from conftest import PKG, ROOT


def declared_functions():
    text = (ROOT / "include" / "srt_amd.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(srt_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for n in ("srt_create", "srt_set_int", "srt_dispatch", "srt_finish", "srt_upload_scene",
              "srt_update_model_matrix", "srt_trace_closest", "srt_render_frames", "srt_model_load"):
        assert n in names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", str(PKG / "libsrt_amd.so")], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing


def test_python_binding_covers_header():
    from srt_amd import _lib

    assert set(declared_functions()) == set(_lib.EXPORTED_SYMBOLS)
    lib = _lib.lib()
    assert lib.srt_abi_version() == 2
    for n in declared_functions():
        assert isinstance(getattr(lib, n), ctypes._CFuncPtr)


def test_record_sizes_match_std430():
    from srt_amd import _lib

    assert ctypes.sizeof(_lib.BvhRecord) == 80
    assert ctypes.sizeof(_lib.BvhNode) == 32
    assert ctypes.sizeof(_lib.MaterialObj) == 48
    assert ctypes.sizeof(_lib.Triangle) == 16
    assert ctypes.sizeof(_lib.Vertex) == 32
    assert ctypes.sizeof(_lib.Light) == 32
    assert ctypes.sizeof(_lib.Ray) == 32


def test_host_entry_points_validate_arguments():
    """Status codes instead of std::terminate / std::runtime_error (no device needed)."""
    from srt_amd import _lib

    lib = _lib.lib()
    assert lib.srt_model_load(None, None) == _lib.SRT_ERR_INVALID
    h = ctypes.c_void_p()
    assert lib.srt_model_load(b"/nonexistent/x.obj", ctypes.byref(h)) == _lib.SRT_ERR_IO
    assert "cannot open" in _lib.last_error()
    assert lib.srt_set_int(None, b"Width", 4) == _lib.SRT_ERR_INVALID
    assert lib.srt_dispatch(None, 1, 1) == _lib.SRT_ERR_INVALID
    assert lib.srt_scene_build(None, 0, None) == _lib.SRT_ERR_INVALID


def test_cpp_host_api_compiles():
    """The C++ mirror of the reference's classes (include/srt/srt.hpp) compiles against the C ABI."""
    src = ROOT / "tests" / "cpp" / "test_api.cpp"
    if not src.exists():
        pytest.skip("no C++ API test source")
    out = ROOT / "tests" / "cpp" / "_build"
    out.mkdir(exist_ok=True)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", str(ROOT / "include"), str(src), "-o",
                    str(out / "test_api"), "-L", str(PKG), "-lsrt_amd", f"-Wl,-rpath,{PKG}"], check=True)
