"""bench.py's host-side bookkeeping (CPU): the per-rank table at N > 1 (each rank's render and exchange
times, its share of the counted rays and its roofline from the 1-GPU counters scaled by that share), and
the wave-cycle split of the second SQ pass.  No GPU: counters and code hash are stubbed."""
import math

import pytest

import bench

CNT = {  # one launch's counters (the metric launch's magnitudes)
    "SQ_INSTS_VALU": 1.2e11, "SQ_THREAD_CYCLES_VALU": 3.3e12, "SQ_LDS_IDX_ACTIVE": 3.9e10,
    "SQ_LDS_BANK_CONFLICT": 1.3e10, "SQ_WAVE_CYCLES": 3.5e11, "SQ_WAIT_ANY": 9.3e10, "SQ_BUSY_CYCLES": 1.1e10,
    "SQ_INSTS_SALU": 3.6e10, "hbm_bytes": 7.0e10, "SQ_ACTIVE_INST_ANY": 1.75e11, "SQ_WAIT_INST_ANY": 8.2e10,
    "SQ_ACTIVE_INST_VALU": 1.26e11, "SQ_ACTIVE_INST_VALU2": 4.3e10, "code_hash": "h", "source": "stub",
}


@pytest.fixture()
def stub(monkeypatch):
    monkeypatch.setattr(bench, "code_hash", lambda: "h")
    monkeypatch.setattr(bench, "load_counters", lambda wl: dict(CNT))


def test_issue_split_sums_to_the_wave_cycles():
    s = bench.issue_split(CNT, 0.1457)
    wc = s["wave_cycles"]
    assert wc["issuing"] + wc["waiting"] + wc["issue_stalled"] == pytest.approx(1.0, abs=0.01)
    # one quad-cycle per instruction: 1.75e11 over 1024 SIMDs x 0.1457 s x 2.4 GHz / 4
    assert s["instructions_per_simd_quad_cycle"] == pytest.approx(1.75e11 / (1024 * 0.1457 * 2.4e9 / 4), rel=1e-3)
    assert bench.issue_split({"SQ_INSTS_VALU": 1.0}, 1.0) == {}


def test_per_rank_lines_scale_the_counters_by_the_ray_share(stub):
    table = [{"kernel_ms": 20.0, "launches_per_step": 1, "overlap": True, "exchange_ms": 0.3, "rays": 300,
              "algorithmic_bytes": 3000},
             {"kernel_ms": 19.0, "launches_per_step": 1, "overlap": True, "exchange_ms": 0.2, "rays": 100,
              "algorithmic_bytes": 1000}]
    ranks = bench.per_rank_lines(table, "rubik_1920x1080_256spp", "k", False)
    assert [r["rays_share"] for r in ranks] == [0.75, 0.25]
    r0, r1 = (r["roofline"] for r in ranks)
    assert r0["counters_scaled_by_ray_share"] == 0.75 and r1["counters_scaled_by_ray_share"] == 0.25
    # a rank's VALU issue: its share of the launch's instructions over its own kernel time
    want0 = 0.75 * CNT["SQ_INSTS_VALU"] / 20e-3 / 1e9 / bench.VALU_PEAK_GIPS
    assert r0["fractions"]["valu_issue"] == pytest.approx(want0, rel=1e-3)
    assert ranks[0]["exchange_ms"] == 0.3 and ranks[1]["kernel_ms"] == 19.0


def test_single_rank_roofline_is_unscaled(stub):
    (r,) = bench.per_rank_lines([{"kernel_ms": 145.7, "launches_per_step": 1, "overlap": True,
                                   "exchange_ms": None, "rays": 918_000_000, "algorithmic_bytes": 2.37e12}],
                                 "rubik_1920x1080_256spp", "k", False)
    rf = r["roofline"]
    assert "counters_scaled_by_ray_share" not in rf and r["rays_share"] == 1.0
    assert rf["bound"] == "valu_issue" and rf["frac"] == pytest.approx(
        CNT["SQ_INSTS_VALU"] / 0.1457 / 1e9 / bench.VALU_PEAK_GIPS, rel=1e-3)
    assert not math.isnan(rf["wave_cycles"]["issue_stalled"])


def test_counters_of_other_code_give_no_roof(monkeypatch):
    monkeypatch.setattr(bench, "code_hash", lambda: "other")
    monkeypatch.setattr(bench, "load_counters", lambda wl: dict(CNT))
    rf = bench.roofline("rubik_1920x1080_256spp", 145.7, 10, "k")
    assert rf["frac"] is None and rf["counters_code_hash"] == "h"


def test_committed_counters_are_for_the_sources():
    """profiles/counters.json must hold counters of the code the sources build: every workload's code_hash
    equals the hash the product build stamps (Makefile `hash`: the preprocessed device translation unit and
    the hipcc flags).  A kernel edit without a re-capture (tools/gpu_round_profiles.sh) would leave the bench line
    without roofs."""
    import json
    import pathlib
    import subprocess

    root = pathlib.Path(__file__).resolve().parent.parent
    want = subprocess.run(["make", "-s", "-C", str(root / "simple-ray-tracer_amd"), "hash"], check=True,
                          capture_output=True, text=True).stdout.strip()
    counters = json.loads((root / "profiles" / "counters.json").read_text())
    assert counters and all(v["code_hash"] == want for v in counters.values()), \
        {k: v["code_hash"] for k, v in counters.items()}


def test_valu_issue_against_the_calibrated_rate(stub):
    """The line also gives the VALU issue against the rate independent f32 arithmetic reaches at the instance's
    occupancy (profiles/r05_calib/valu_issue_calibration.json, tools/valu_issue_probe.hip): the 4-wave LDS kernel
    against the 4-wave rate, a 5-wave instance against the next measured occupancy (8)."""
    rf = bench.roofline("rubik_1920x1080_256spp", 145.7, 10, bench.KERNEL_LDS)
    cal = rf["valu_issue_calibrated"]
    assert cal["waves_per_simd"] == 4 and cal["peak"] < bench.VALU_PEAK_GIPS
    assert cal["frac"] == pytest.approx(rf["fractions"]["valu_issue"] * bench.VALU_PEAK_GIPS / cal["peak"], rel=1e-3)
    g = bench.roofline("torusknot262144out_1920x1080_64spp", 26.2, 10,
                       "srt::sample_kernel<...> (global-scene mode, fused sub-steps, 5 waves per SIMD)", global_mode=True)
    assert g["valu_issue_calibrated"]["waves_per_simd"] == 5 and "8 waves" in g["valu_issue_calibrated"]["basis"]


def test_code_hash_ignores_prose_but_not_code(tmp_path):
    """the code hash is the preprocessed translation unit of pathtrace.hip (comments and
    blank lines gone) plus the hipcc flags, so a comment edit in include/srt_amd.h or a kernel header leaves it
    alone, while a code edit changes it (and counters of other code are then rejected, test above)."""
    import pathlib
    import shutil
    import subprocess

    root = pathlib.Path(__file__).resolve().parent.parent
    pkg = tmp_path / "pkg"
    shutil.copytree(root / "simple-ray-tracer_amd" / "csrc", pkg / "csrc")
    shutil.copy(root / "simple-ray-tracer_amd" / "Makefile", pkg / "Makefile")
    shutil.copytree(root / "include", tmp_path / "include")

    def h():
        return subprocess.run(["make", "-s", "-C", str(pkg), "hash"], check=True, capture_output=True,
                              text=True).stdout.strip()

    base = h()
    assert len(base) == 16 and base != "pp-failed"
    hdr = tmp_path / "include" / "srt_amd.h"
    hdr.write_text(hdr.read_text().replace("/* Closest-hit query:", "/* Closest-hit query (reworded):\n\n *"))
    trav = pkg / "csrc" / "traversal.hpp"
    trav.write_text("// a new comment line\n" + trav.read_text())
    assert h() == base
    k = pkg / "csrc" / "kernels.hpp"
    k.write_text(k.read_text().replace("mk(0.05f, 0.05f, 0.05f)", "mk(0.05f, 0.05f, 0.06f)", 1))
    assert h() != base
