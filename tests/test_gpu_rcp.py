"""Exhaustive check of the triangle test's reciprocal (pathtrace.hip recip_normal).

The kernel replaces the reference's correctly rounded f = 1.0 / a
(ray_intersects.glsl:61-96) with v_rcp_f32 + one FMA Newton step for
2^-126 <= |a| < 2^126 and keeps the division elsewhere.  This runs all 2^32
fp32 inputs on the GPU and requires every mismatch to lie outside that range
(exponent field 0, 253, 254 or 255).
"""
import re
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_newton_reciprocal_is_correctly_rounded(tmp_path):
    exe = tmp_path / "rcp_exhaustive"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
                    "-Wno-unused-value", "-Wno-unused-result", str(ROOT / "tools" / "rcp_exhaustive.hip"),
                    "-o", str(exe)], check=True)
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout + res.stderr
    buckets = [int(m) for m in re.findall(r"^exp\s+(\d+)", res.stdout, re.M)]
    assert set(buckets) <= {0, 253, 254, 255}, res.stdout
    assert "TOTAL" in res.stdout
