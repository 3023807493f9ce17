#!/usr/bin/env python
"""Reduces tools/c2_study.sh's runs (gpurun_out/c2s/b<N>/) into profiles/r04_c2_study.json: for each
sphere_kernel occupancy (blocks per CU), the timed launch's kernel time and its counters, per launch.

  valu_issue      SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x kernel time x 2.4 GHz)
  lane_util       SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU)
  wait_any        SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt)
  wait_inst       SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls)
  l2_hit          TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  fetch_lines_B   2 x FETCH_SIZE (128-B line requests tallied at 64 B on gfx950), per launch and per sample
  write_B         WRITE_SIZE, per launch and per sample (a sample's record is 16 B)
usage: python tools/c2_study.py gpurun_out/c2s [--out profiles/r04_c2_study.json]
"""
from __future__ import annotations

import csv
import json
import pathlib
import sys

CLOCK = 2.4e9
SIMDS = 1024
KERNEL = "void srt::sphere_kernel<false>"


def counters(d: pathlib.Path) -> dict:
    out = {}
    for sub in ("pmc_sq", "pmc_sq2", "pmc_fetch", "pmc_write", "pmc_tcc", "pmc_tcp"):
        p = d / sub / "run_counter_collection.csv"
        if not p.exists():
            continue
        rows = [r for r in csv.DictReader(open(p)) if r["Kernel_Name"].startswith(KERNEL)]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        if not ids:
            continue
        last = ids[-1]  # the timed launch (the counting run is sphere_kernel<true>)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main():
    root = pathlib.Path(sys.argv[1])
    outp = pathlib.Path(sys.argv[sys.argv.index("--out") + 1]) if "--out" in sys.argv else \
        pathlib.Path(__file__).resolve().parents[1] / "profiles" / "r04_c2_study.json"
    res = {"workload": "spheres_1024x1024_64spp_depth4 (C2), sphere_kernel<false>, one timed launch per pass",
           "by_blocks": {}}
    for d in sorted(root.glob("b*")):
        n = int(d.name[1:])
        bench = json.loads((d / "bench.json").read_text())
        k_ms = bench["roofline"]["kernel_ms"]
        c = counters(d)
        samples = 1024 * 1024 * 64
        e = {"blocks_per_cu": n, "waves_per_simd": n, "kernel_ms": k_ms, "Mrays_s": bench["value"],
             "code_hash": bench["code_hash"], "counters": c}
        ks = k_ms * 1e-3
        if "SQ_INSTS_VALU" in c:
            e["valu_issue"] = c["SQ_INSTS_VALU"] * 2 / (SIMDS * ks * CLOCK)
            e["lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_INSTS_VALU"])
            e["wait_any"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_INST_ANY" in c:
            e["wait_inst"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in c else None
        if "TCC_HIT_sum" in c:
            e["l2_hit"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1.0)
        if "FETCH_SIZE" in c:
            e["fetch_lines_B"] = 2 * c["FETCH_SIZE"] * 1024
            e["fetch_lines_B_per_sample"] = e["fetch_lines_B"] / samples
        if "WRITE_SIZE" in c:
            e["write_B"] = c["WRITE_SIZE"] * 1024
            e["write_B_per_sample"] = e["write_B"] / samples
        res["by_blocks"][str(n)] = e
    outp.write_text(json.dumps(res, indent=1) + "\n")
    keys = ("kernel_ms", "valu_issue", "lane_util", "wait_any", "wait_inst", "l2_hit", "fetch_lines_B_per_sample",
            "write_B_per_sample")
    print("blocks " + " ".join(keys))
    for n, e in res["by_blocks"].items():
        print(n, " ".join(f"{e.get(k, float('nan')):.4g}" if isinstance(e.get(k), (int, float)) else "-" for k in keys))


if __name__ == "__main__":
    main()
