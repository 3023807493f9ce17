#!/usr/bin/env python
"""Reduces a counter study's runs into JSON: tools/probes/c2_study.sh (gpurun_out/c2s/b<N>/, one per
sphere_kernel occupancy) or tools/pmc_study.sh (gpurun_out/<name>/<variant>/, --kernel PREFIX): for each,
the timed launch's kernel time and its counters, per launch.

  valu_issue      SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x kernel time x 2.4 GHz)
  lane_util       SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU)
  wait_any        SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt)
  wait_inst       SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls)
  valu_busy       cycle-weighted: 4 x SQ_ACTIVE_INST_VALU (quad-cycles waves spend executing VALU instructions)
                  / (1024 SIMDs x the pass's cycles, GRBM_GUI_ACTIVE / 8 XCDs): a slow instruction weighs its cycles
  valu2_share     SQ_ACTIVE_INST_VALU2 / SQ_ACTIVE_INST_VALU (quad-cycles in which two VALU instructions issue)
  cycles_per_valu 4 x SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU (2 for a plain wave64 instruction)
  l2_hit          TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  fetch_lines_B   2 x FETCH_SIZE (128-B line requests tallied at 64 B on gfx950), per launch and per sample
  write_B         WRITE_SIZE, per launch and per sample (a sample's record is 16 B)
usage: python tools/c2_study.py gpurun_out/c2s [--out profiles/r04_c2_study.json]
       python tools/c2_study.py gpurun_out/torus --kernel "void srt::sample_kernel<false" --out ...
"""
from __future__ import annotations

import csv
import json
import pathlib
import sys

CLOCK = 2.4e9
SIMDS = 1024
KERNEL = "void srt::sphere_kernel<false>"


VMEM_PASSES = ("pmc_ta1", "pmc_ta2", "pmc_td", "pmc_tcp1", "pmc_tcp2", "pmc_tcp3")  # tools/vmem_study.sh


def counters(d: pathlib.Path, kernel: str = KERNEL, per_pass: dict | None = None) -> dict:
    """The timed launch's counters, merged over the passes (GRBM_GUI_ACTIVE from the first pass holding it;
    `per_pass` receives each pass's own counters, for ratios against that pass's cycles)."""
    out = {}
    for sub in ("pmc_sq", "pmc_sq2", "pmc_cyc", "pmc_fetch", "pmc_write", "pmc_tcc", "pmc_tcp") + VMEM_PASSES:
        p = d / sub / "run_counter_collection.csv"
        if not p.exists():
            continue
        rows = [r for r in csv.DictReader(open(p)) if r["Kernel_Name"].startswith(kernel)]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        if not ids:
            continue
        last = ids[-1]  # the timed launch (the counting run is sphere_kernel<true>)
        mine = {}
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                mine[r["Counter_Name"]] = mine.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if per_pass is not None:
            per_pass[sub] = mine
        for k, v in mine.items():
            if k == "GRBM_GUI_ACTIVE" and k in out:
                continue
            out[k] = v
    return out


CUS = 256


def vmem_ratios(pp: dict) -> dict:
    """Vector-memory pipeline shares per pass (each against its own cycles, GRBM_GUI_ACTIVE / 8 XCDs):
    ta_busy / td_busy (TA_TA_BUSY, TD_TD_BUSY over 256 CUs x cycles), the TA's cycles stalled on the
    TCP for addresses / data, TD stalled on the TC, the mean L1 -> L2 read latency (cycles per request),
    the UTCL1 translation miss rate and the TCP's stall shares."""
    e = {}

    def cyc(sub):
        return pp.get(sub, {}).get("GRBM_GUI_ACTIVE", 0.0) / 8.0

    ta1, ta2, td = pp.get("pmc_ta1", {}), pp.get("pmc_ta2", {}), pp.get("pmc_td", {})
    if ta1 and cyc("pmc_ta1"):
        e["ta_busy"] = ta1["TA_TA_BUSY_sum"] / (CUS * cyc("pmc_ta1"))
        e["ta_addr_stalled_by_tc"] = ta1["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / max(ta1["TA_TA_BUSY_sum"], 1.0)
    if ta2 and cyc("pmc_ta2"):
        e["ta_data_stalled_by_tc"] = ta2["TA_DATA_STALLED_BY_TC_CYCLES_sum"] / (CUS * cyc("pmc_ta2"))
        e["ta_flat_read_wavefronts"] = ta2["TA_FLAT_READ_WAVEFRONTS_sum"]
    if td and cyc("pmc_td"):
        e["td_busy"] = td["TD_TD_BUSY_sum"] / (CUS * cyc("pmc_td"))
        e["td_tc_stall"] = td["TD_TC_STALL_sum"] / (CUS * cyc("pmc_td"))
    t1, t2, t3 = pp.get("pmc_tcp1", {}), pp.get("pmc_tcp2", {}), pp.get("pmc_tcp3", {})
    if t1:
        e["l2_read_latency_cyc"] = t1["TCP_TCC_READ_REQ_LATENCY_sum"] / max(t1["TCP_TCC_READ_REQ_sum"], 1.0)
        e["tcp_pending_stall_cyc"] = t1["TCP_PENDING_STALL_CYCLES_sum"]
        e["tcp_tcr_stall_cyc"] = t1["TCP_TCR_TCP_STALL_CYCLES_sum"]
    if t2:
        e["utcl1_miss_rate"] = t2["TCP_UTCL1_TRANSLATION_MISS_sum"] / max(t2["TCP_UTCL1_REQUEST_sum"], 1.0)
        e["tcp_read_tagconflict_stall_cyc"] = t2["TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"]
    if t3:
        e["tcp_latency_cyc_per_access"] = t3["TCP_TCP_LATENCY_sum"] / max(t3["TCP_TOTAL_CACHE_ACCESSES_sum"], 1.0)
        e["tcp_ta_data_stall_cyc"] = t3["TCP_TCP_TA_DATA_STALL_CYCLES_sum"]
        e["tcp_accesses"] = t3["TCP_TOTAL_CACHE_ACCESSES_sum"]
    return e


def main():
    root = pathlib.Path(sys.argv[1])
    outp = pathlib.Path(sys.argv[sys.argv.index("--out") + 1]) if "--out" in sys.argv else \
        pathlib.Path(__file__).resolve().parents[1] / "profiles" / "r04_c2_study.json"
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else KERNEL
    study = "--kernel" in sys.argv
    res = {"workload": "spheres_1024x1024_64spp_depth4 (C2), sphere_kernel<false>, one timed launch per pass"
           if not study else f"{root.name}: {kernel}..., one timed launch per pass", "by_blocks": {}}
    for d in sorted(p for p in root.iterdir() if p.is_dir()):
        n = d.name[1:] if not study else d.name
        bench = json.loads((d / "bench.json").read_text())
        k_ms = bench["roofline"]["kernel_ms"]
        pp = {}
        c = counters(d, kernel, pp)
        cfg = bench["config"]
        samples = cfg["width"] * cfg["height"] * cfg["spp"]
        e = {"variant": n, "kernel_ms": k_ms, "Mrays_s": bench["value"], "rays": bench["rays_per_step"],
             "code_hash": bench["code_hash"], "counters": c}
        ks = k_ms * 1e-3
        if "SQ_INSTS_VALU" in c:
            e["valu_issue"] = c["SQ_INSTS_VALU"] * 2 / (SIMDS * ks * CLOCK)
            e["lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_INSTS_VALU"])
            e["wait_any"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        if "SQ_ACTIVE_INST_VALU" in c and "GRBM_GUI_ACTIVE" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / 8.0  # (the pass's own cycles; summed over the 8 XCDs)
            e["valu_busy"] = 4.0 * c["SQ_ACTIVE_INST_VALU"] / (SIMDS * cyc)
            e["valu2_share"] = c.get("SQ_ACTIVE_INST_VALU2", 0.0) / max(c["SQ_ACTIVE_INST_VALU"], 1.0)
            e["sca_busy"] = 4.0 * c.get("SQ_ACTIVE_INST_SCA", 0.0) / (SIMDS * cyc)
            if "SQ_INSTS_VALU" in c:
                e["cycles_per_valu"] = 4.0 * c["SQ_ACTIVE_INST_VALU"] / c["SQ_INSTS_VALU"]
                e["trans_share"] = c.get("SQ_INSTS_VALU_TRANS_F32", 0.0) / c["SQ_INSTS_VALU"]
                e["f64_share"] = (c.get("SQ_INSTS_VALU_MUL_F64", 0.0) + c.get("SQ_INSTS_VALU_FMA_F64", 0.0)) / c["SQ_INSTS_VALU"]
        if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
            e["wait_inst"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
            e["active_inst"] = c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"] if "SQ_ACTIVE_INST_ANY" in c else None
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS"):
            if k in c:
                e[k.lower() + "_per_ray"] = c[k] / bench["rays_per_step"]
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
            e["l1_miss_req_frac"] = c["TCP_TCC_READ_REQ_sum"] / max(c["TCP_TOTAL_CACHE_ACCESSES_sum"], 1.0)
        if "TCC_HIT_sum" in c:
            e["l2_hit"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1.0)
        if "FETCH_SIZE" in c:
            e["fetch_lines_B"] = 2 * c["FETCH_SIZE"] * 1024
            e["fetch_lines_B_per_sample"] = e["fetch_lines_B"] / samples
        if "WRITE_SIZE" in c:
            e["write_B"] = c["WRITE_SIZE"] * 1024
            e["write_B_per_sample"] = e["write_B"] / samples
        e.update(vmem_ratios(pp))
        if "tcp_accesses" in e and "SQ_INSTS_VMEM_RD" in c:
            e["tcp_accesses_per_vmem_rd"] = e["tcp_accesses"] / max(c["SQ_INSTS_VMEM_RD"], 1.0)
        res["by_blocks"][str(n)] = e
    outp.write_text(json.dumps(res, indent=1) + "\n")
    keys = ("kernel_ms", "valu_issue", "valu_busy", "cycles_per_valu", "valu2_share", "sca_busy", "trans_share",
            "f64_share", "lane_util", "wait_any", "wait_inst", "active_inst", "l2_hit",
            "l1_miss_req_frac", "fetch_lines_B_per_sample", "write_B_per_sample", "sq_insts_valu_per_ray",
            "sq_insts_salu_per_ray", "sq_insts_vmem_rd_per_ray", "sq_insts_lds_per_ray", "ta_busy",
            "ta_addr_stalled_by_tc", "ta_data_stalled_by_tc", "td_busy", "td_tc_stall", "l2_read_latency_cyc",
            "utcl1_miss_rate", "tcp_latency_cyc_per_access", "tcp_accesses_per_vmem_rd")
    print("blocks " + " ".join(keys))
    for n, e in res["by_blocks"].items():
        print(n, " ".join(f"{e.get(k, float('nan')):.4g}" if isinstance(e.get(k), (int, float)) else "-" for k in keys))


if __name__ == "__main__":
    main()
