#!/usr/bin/env python3
"""Throughput time per launch of a kernel from a rocprofv3 kernel trace: the check of bench.py's kernel_ms.

Overlapped sample launches (pipeline slots) are dispatched while other launches
still hold the CUs (the hardware may also run two slots' launches side by side, or the later one first),
so a dispatch's Start..End includes its wait for them.  bench.py's kernel time is the union of the
launches' own spans (srt_kernel_time); here the same union is taken over the trace's timestamps: in start
order, launch k adds the part of [Start_k, End_k] after the latest end so far -- the interval between
consecutive launch ends when launches overlap, the dispatch's duration when they run in series.

  python tools/trace_intervals.py <run_kernel_trace.csv> <kernel-name substring> [last N] [bench line json]

Prints one JSON object: the dispatches matched, the last N of them (the timed region: the bench's first
dispatch of a timed instance is its warmup), their mean dispatch duration (what --stats averages), their
mean throughput time, and, given the bench line, its kernel_ms and the relative difference.
"""
from __future__ import annotations

import csv
import json
import sys


def throughput_ms(rows) -> list[float]:
    """Per launch, in start order: what it adds to the union of the dispatches' intervals, in ms."""
    out, prev_end = [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        t0 = s if prev_end is None else max(s, min(prev_end, e))
        out.append((e - t0) * 1e-6)
        prev_end = e if prev_end is None else max(prev_end, e)
    return out


def main(argv):
    path, pat = argv[1], argv[2]
    last = int(argv[3]) if len(argv) > 3 else 0
    with open(path, newline="") as f:
        rows = [r for r in csv.DictReader(f) if pat in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if not rows:
        raise SystemExit(f"no dispatch of a kernel matching {pat!r}")
    thr = throughput_ms(rows)  # (the interval of the region's first launch counts from its predecessor's end)
    if last:
        rows, thr = rows[-last:], thr[-last:]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]
    res = {"trace": path, "kernel": rows[0]["Kernel_Name"][:160], "dispatches": len(rows),
           "mean_dispatch_duration_ms": round(sum(dur) / len(dur), 4),
           "mean_throughput_ms": round(sum(thr) / len(thr), 4),
           "throughput_ms": [round(x, 4) for x in thr]}
    if len(argv) > 4:
        with open(argv[4]) as f:
            line = json.loads([l for l in f if l.startswith("{")][-1])
        k = line["roofline"]["kernel_ms"]
        res["bench_kernel_ms"] = k
        res["relative_difference"] = round(res["mean_throughput_ms"] / k - 1.0, 5)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv)
