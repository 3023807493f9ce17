"""Writes profiles/traffic.json from a round's FETCH_SIZE / WRITE_SIZE passes (tools/profile_round.sh).

usage: python tools/traffic_json.py gpurun_out/r01 [workload]
HBM bytes per launch of the timed sample kernel = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(MI355X_MICROARCH.md, HBM section: gfx950 FETCH_SIZE counts 128-B requests as 64 B).
"""
import csv
import json
import pathlib
import sys

out_dir = pathlib.Path(sys.argv[1])
workload = sys.argv[2] if len(sys.argv) > 2 else "rubik_1920x1080_256spp"


def counter(name, sub):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(out_dir / sub / "run_counter_collection.csv"))
            if r["Kernel_Name"].startswith("void srt::sample_kernel<false") and r["Counter_Name"] == name]
    assert vals, f"no sample_kernel<false ...> row for {name} in {sub}"
    return vals[-1]


fetch_kb = counter("FETCH_SIZE", "pmc_fetch")
write_kb = counter("WRITE_SIZE", "pmc_write")
root = pathlib.Path(__file__).resolve().parent.parent
p = root / "profiles" / "traffic.json"
data = json.loads(p.read_text()) if p.exists() else {}
data[workload] = {
    "hbm_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024,
    "fetch_size_kb": fetch_kb,
    "write_size_kb": write_kb,
    "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024: MI355X_MICROARCH.md 'HBM' -- gfx950 FETCH_SIZE tallies "
                  "128-B requests at 64 B (x2); WRITE_SIZE exact for 16-B stores. The sample kernel's reads are 4-8 B "
                  "noise gathers (uncalibrated width), so the x2 makes this an upper bound.",
    "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, python bench.py --steps 1 ({out_dir.name})",
}
p.write_text(json.dumps(data, indent=1) + "\n")
print(json.dumps(data[workload], indent=1))
