"""Joins tools/gather_calib.sh's timing run and PMC passes into profiles/r03_gather_calibration.json.

usage: python tools/gather_calib.py gpurun_out/calib

Per case (access pattern x table size): algorithmic read bytes of one launch, its time, and what the
memory-side counters report for it -- FETCH_SIZE x 1024, TCC_EA0_RDREQ_DRAM_32B x 32, the request
counts -- as ratios to the algorithmic bytes.  The calibration factor a kernel with this access pattern
should use to turn FETCH_SIZE into bytes moved is fetch_factor = (bytes the pattern moves) / (FETCH_SIZE
x 1024): 2 for wide streaming reads (MI355X_MICROARCH.md 'HBM').
"""
import csv
import json
import pathlib
import sys
from collections import defaultdict

d = pathlib.Path(sys.argv[1])
root = pathlib.Path(__file__).resolve().parent.parent


def timing(path):
    rows = []
    for line in path.read_text().splitlines():
        f = line.split()
        if len(f) != 7 or f[0] not in ("stream", "rec32", "rec48", "rec64", "rec128"):
            continue
        name, T, rep, b, wb, ms, gbs = f
        rows.append(dict(case=name, table_bytes=int(T), rep=int(rep), bytes=int(b), write_bytes=int(wb),
                         ms=float(ms), GBps=float(gbs)))
    return rows


def counters(sub):
    """[{counter: value}] per non-fill dispatch, in dispatch order."""
    p = next((d / sub).rglob("*counter_collection.csv"))
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(p)):
        did = int(r["Dispatch_Id"])
        names[did] = r["Kernel_Name"]
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
    return [dict(per[k]) for k in sorted(per) if "fill_kernel" not in names[k]]


t3 = timing(d / "timing.txt")
t1 = timing(d / "pmc_fetch.log")  # the one-rep run the passes profiled (same launches, same order)
fetch, req, tcc = counters("pmc_fetch"), counters("pmc_req"), counters("pmc_tcc")
assert len(fetch) == len(req) == len(tcc) == len(t1), (len(fetch), len(req), len(tcc), len(t1))
out = []
for i, c in enumerate(t1):
    best = min((r for r in t3 if r["case"] == c["case"] and r["table_bytes"] == c["table_bytes"]),
               key=lambda r: r["ms"])
    f = fetch[i]["FETCH_SIZE"] * 1024
    dram = req[i]["TCC_EA0_RDREQ_DRAM_32B"] * 32
    hits, miss = tcc[i].get("TCC_HIT_sum", 0.0), tcc[i].get("TCC_MISS_sum", 0.0)
    out.append({
        "case": c["case"], "table_MiB": c["table_bytes"] >> 20, "algorithmic_bytes": c["bytes"],
        "ms": best["ms"], "GBps": round(c["bytes"] / (best["ms"] * 1e-3) / 1e9, 1),
        "fetch_size_bytes": f, "fetch_over_algorithmic": round(f / c["bytes"], 4),
        "dram_32B_bytes": dram, "dram_32B_over_algorithmic": round(dram / c["bytes"], 4),
        "rdreq": req[i]["TCC_EA0_RDREQ_sum"], "rdreq_32B": req[i]["TCC_EA0_RDREQ_32B_sum"],
        "bubble_128B": req[i]["TCC_BUBBLE_sum"],
        "tcc_hit_rate": round(hits / max(hits + miss, 1.0), 4),
    })
    print(f"{c['case']:7s} {c['table_bytes'] >> 20:5d} MiB  {out[-1]['GBps']:8.1f} GB/s  FETCH/alg "
          f"{out[-1]['fetch_over_algorithmic']:.3f}  DRAM32B/alg {out[-1]['dram_32B_over_algorithmic']:.3f}  "
          f"rdreq {req[i]['TCC_EA0_RDREQ_sum']:.3g} 32B {req[i]['TCC_EA0_RDREQ_32B_sum']:.3g} "
          f"bubble {req[i]['TCC_BUBBLE_sum']:.3g}  L2 hit {out[-1]['tcc_hit_rate']:.3f}")
res = {"tool": "tools/gather_calib.hip + tools/gather_calib.sh (rocprofv3 --pmc passes) + tools/gather_calib.py",
       "note": "one launch per case reads ~1 GiB of whole random records (or streams the table once) with "
               "16 waves per CU; GBps = algorithmic bytes / best of 3 timed launches",
       "cases": out}
(root / "profiles" / "r03_gather_calibration.json").write_text(json.dumps(res, indent=1) + "\n")
