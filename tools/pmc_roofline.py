"""Writes profiles/counters.json from a round's rocprofv3 PMC passes (tools/profile_round.sh).

usage: python tools/pmc_roofline.py gpurun_out/r02 [--tag r02] [--workload NAME]
(--workload: a single-leg run, e.g. tools/pmc_c5.sh's, whose global-scene instance is NAME; --il: that
run took the IL-pattern instance, as trees past 600 MB do; --sum: sum every non-counting sample_kernel
(or sphere_kernel) dispatch of a single-workload run, whatever its instance, e.g. tools/pmc_configs.sh's
C2 and C4)

Each pass ran `python bench.py --steps 1 --warmup 0 --no-cpu-baseline`, so every leg's timed step
launched its sample_kernel<false, ...> instance exactly once (the counting run is the <true, ...>
instance).  Per leg and launch:
  SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU, SQ_LDS_IDX_ACTIVE, SQ_LDS_BANK_CONFLICT, SQ_WAVE_CYCLES,
  SQ_WAIT_ANY, SQ_BUSY_CYCLES, SQ_INSTS_SALU, GRBM_GUI_ACTIVE  (one SQ pass)
  hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024  (separate passes; MI355X_MICROARCH.md 'HBM':
              gfx950 FETCH_SIZE tallies 128-B requests at 64 B, WRITE_SIZE is exact for 16-B stores)
bench.py divides these by its live kernel time (HIP events) to report the roofs.
"""
import csv
import json
import pathlib
import sys

out_dir = pathlib.Path(sys.argv[1])
tag = sys.argv[sys.argv.index("--tag") + 1] if "--tag" in sys.argv else out_dir.name
only = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else None
root = pathlib.Path(__file__).resolve().parent.parent

AIRPLANE_LEG = "torusknot262144_airplane_materials_1920x1080_256spp"  # bench.py's texture-sampling leg (C3's spp)
LEGS = {  # kernel instance -> the workloads bench.py runs on it, in launch order (one timed launch each)
    "void srt::sample_kernel<false, true, true, 1024, false, false, 4>": ["rubik_1920x1080_256spp"],
    "void srt::sample_kernel<false, false, true, 256, false, true, 4>": ["synthetic1000000_1920x1080_16spp"],
    "void srt::sample_kernel<false, false, true, 256, false, true, 5>": ["torusknot262144out_1920x1080_64spp"],
    "void srt::sample_kernel<false, false, true, 256, true, true, 5>": [AIRPLANE_LEG],
}


if only:  # the one timed global-scene instance of the run, whatever its waves per SIMD
    LEGS = {"void srt::sample_kernel<false, false, true, 256, false, " + ("false," if "--il" in sys.argv else "true,"): [only]}
# --sum: a single-workload run whose timed step may be several launches (sample-buffer chunks, e.g. C4):
# the counters of every non-counting sample_kernel dispatch are summed (bench's kernel_ms sums the same
# launches' HIP-event times); the counting run is the <true, ...> instance and is left out.
SUM = "--sum" in sys.argv
if SUM:
    assert only, "--sum needs --workload"
    LEGS = {("void srt::sample_kernel<false, ", "void srt::sphere_kernel<false>"): [only]}


def rows(sub):
    p = out_dir / sub / "run_counter_collection.csv"
    return list(csv.DictReader(open(p)))


def per_launch(sub):
    """{workload: {counter: value}} of each leg's dispatch (summed over the dimensions rocprofv3 splits)."""
    out = {}
    for leg_kernel, wls in LEGS.items():
        rs = [r for r in rows(sub) if r["Kernel_Name"].startswith(leg_kernel)]  # (str.startswith takes a tuple)
        if SUM:
            agg = {}
            for r in rs:
                agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            out[wls[0]] = agg
            continue
        ids = sorted({int(r["Dispatch_Id"]) for r in rs})
        for wl, did in zip(wls, ids[-len(wls):] if len(ids) >= len(wls) else ids):
            agg = {}
            for r in rs:
                if int(r["Dispatch_Id"]) == did:
                    agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            out[wl] = agg
    return out


def bench_code_hash(sub):
    """code_hash of the library the pass profiled: bench.py's JSON line in the pass's log (<sub>.log)."""
    hashes = set()
    for line in (out_dir / f"{sub}.log").read_text().splitlines():
        if line.startswith("{"):
            d = json.loads(line)
            hashes |= {d["roofline"].get("code_hash")} | {l["roofline"].get("code_hash") for l in d.get("legs", [])}
    hashes.discard(None)
    assert len(hashes) == 1, f"{sub}.log: code hashes {hashes}"
    return hashes.pop()


sq, fetch, write = per_launch("pmc_sq"), per_launch("pmc_fetch"), per_launch("pmc_write")
code = {bench_code_hash(s) for s in ("pmc_sq", "pmc_fetch", "pmc_write") + (("pmc_sq2",) if (out_dir / "pmc_sq2").exists() else ())}
assert len(code) == 1, f"the passes profiled different code: {code}"
code = code.pop()
p = root / "profiles" / "counters.json"
data = json.loads(p.read_text()) if p.exists() else {}
for wl in sq:
    d = dict(sq[wl])
    d["FETCH_SIZE"] = fetch[wl]["FETCH_SIZE"]
    d["WRITE_SIZE"] = write[wl]["WRITE_SIZE"]
    d["hbm_bytes"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
    if (out_dir / "pmc_sq2").exists():  # issue and wave-state counters (tools/profile_round.sh's second SQ pass)
        d.update({k: v for k, v in per_launch("pmc_sq2").get(wl, {}).items() if k not in d})
    if (out_dir / "pmc_tcc").exists():
        tcc = per_launch("pmc_tcc").get(wl, {})
        d.update({k: v for k, v in tcc.items()})
    d["source"] = (f"rocprofv3 --pmc passes ({tag}): SQ counters + GRBM_GUI_ACTIVE, FETCH_SIZE, WRITE_SIZE; "
                   f"python bench.py --steps 1 --warmup 0 --no-cpu-baseline; per launch of the timed step")
    d["code_hash"] = code
    data[wl] = d
    lane = d["SQ_THREAD_CYCLES_VALU"] / (64 * d["SQ_INSTS_VALU"])
    print(f"{wl}: VALU {d['SQ_INSTS_VALU']:.4g} insts, lane util {lane:.3f}, LDS active {d['SQ_LDS_IDX_ACTIVE']:.4g}, "
          f"conflict {d['SQ_LDS_BANK_CONFLICT'] / max(d['SQ_LDS_IDX_ACTIVE'], 1):.3f}, HBM {d['hbm_bytes'] / 1e9:.2f} GB, "
          f"wait {d['SQ_WAIT_ANY'] / d['SQ_WAVE_CYCLES']:.3f}")
p.write_text(json.dumps(data, indent=1) + "\n")
