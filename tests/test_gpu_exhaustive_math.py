"""Exhaustive checks (all 2^32 fp32 inputs, on the GPU) of the kernel's fast exact arithmetic.

* recip_normal (csrc/traversal.hpp): the triangle test's f = 1.0 / a (ray_intersects.glsl:61-96)
  as v_rcp_f32 + one FMA Newton step for 2^-126 <= |a| < 2^126, the division elsewhere.
  Every mismatch against the correctly rounded quotient must lie outside that range
  (exponent field 0, 253, 254 or 255).
* pow5_f (pt_math.hpp): the contract's pow(x, 5.0) (brdf.glsl:34-41) must equal x^5 rounded
  to nearest-even, from its exact integer value, for every input with a normal result.
"""
import re
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

HIPCC = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
         "-Wno-unused-value", "-Wno-unused-result", "-I", str(ROOT / "simple-ray-tracer_amd" / "csrc")]


def _run(tool, tmp_path):
    exe = tmp_path / tool
    subprocess.run(HIPCC + [str(ROOT / "tools" / f"{tool}.hip"), "-o", str(exe)], check=True)
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    return res.stdout


def test_newton_reciprocal_is_correctly_rounded(tmp_path):
    out = _run("rcp_exhaustive", tmp_path)
    buckets = [int(m) for m in re.findall(r"^exp\s+(\d+)", out, re.M)]
    assert set(buckets) <= {0, 253, 254, 255}, out
    assert "TOTAL" in out


def test_pow5_is_correctly_rounded(tmp_path):
    out = _run("pow5_exhaustive", tmp_path)
    m = re.search(r"EXACT_MISMATCH (\d+) CHECKED (\d+)", out)
    assert m and int(m.group(1)) == 0 and int(m.group(2)) > 400_000_000, out
