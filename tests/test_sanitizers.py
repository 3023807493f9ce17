"""The host side under AddressSanitizer + UBSan: tools/san_tests.sh builds the C ABI /
host producers (libsrt_amd_san.so) and the oracle (liboracle_san.so) instrumented and reruns the CPU tests
that drive them -- OBJ/MTL parsing, BVH builds (serial and threaded), noise, camera state, output stage,
oracle math and renders -- with the sanitizer runtimes preloaded; any report aborts the run."""
from __future__ import annotations

import os
import subprocess

from conftest import ROOT

SUITES = ["tests/test_producers.py", "tests/test_interactive.py", "tests/test_oracle_pins.py",
          "tests/test_output_stage.py", "tests/test_airplane_materials.py", "tests/test_abi.py"]


def test_cpu_suites_clean_under_asan_ubsan():
    env = dict(os.environ)
    res = subprocess.run(["bash", str(ROOT / "tools" / "san_tests.sh"), *SUITES], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=900)
    assert res.returncode == 0, res.stdout[-4000:] + res.stderr[-4000:]
    assert " passed" in res.stdout
