"""bench.py's line on the GPU (a short run): C3's regime beside the headline and every workload's ray mix.

VERDICT r05 items 2 and 4: the line carries `c3_regime` (the Airplane-material leg: C3's frame and material
path in global-scene mode, which the absent Airplane OBJ would take) with its own roofline, and each workload
its `ray_kinds` (camera, shadow, bounce rays of the counting launch, srt_ray_kinds), which sum to its rays.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_line_carries_c3_regime_and_ray_kinds():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, str(ROOT / "bench.py"), "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
           "--width", "320", "--height", "180", "--spp", "4", "--no-global-leg", "--surface-spp", "2",
           "--airplane-spp", "2"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    line = json.loads([l for l in res.stdout.splitlines() if l.startswith("{")][-1])
    legs = {l["leg"]: l for l in line["legs"]}
    assert set(legs) == {"surface_mesh", "airplane_materials"}
    for wl in [line] + line["legs"]:
        k = wl["ray_kinds"]
        assert k["camera"] + k["shadow"] + k["bounce"] == wl["rays_per_step"]
    assert line["ray_kinds"]["camera"] == 320 * 180 * 4
    air = legs["airplane_materials"]
    assert air["config"]["spp"] == 2 and air["ray_kinds"]["camera"] == 1920 * 1080 * 2
    c3 = line["c3_regime"]
    assert c3["workload"] == air["workload"] and c3["value"] == air["value"] > 0
    assert c3["ms_per_step"] == air["ms_per_step"] and c3["spp"] == 2 and c3["roofline"] == air["roofline"]
    # the surface-mesh leg is the outward knot: its paths bounce
    assert legs["surface_mesh"]["workload"].startswith("torusknot262144out_")
    assert legs["surface_mesh"]["ray_kinds"]["bounce_share"] > 0.2
