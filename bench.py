#!/usr/bin/env python
"""bench.py -- Mrays/s of the MI355X path tracer on BASELINE.json's metric workload.

BASELINE metric: "Mrays/s + frame ms at 1920x1080, 256 spp, Airplane OBJ; 1/2/4/8 GPU".
The Airplane OBJ is absent from the reference checkout (.MISSING_LARGE_BLOBS), so
the default workload is the same frame shape and sampling on the reference's
shipped model scene (Rubik.obj, model camera, the 6 lights of src/main.cpp:584-589).

A step = one full progressive render of the workload: the reset frame + `spp`
sampled frames (one fused kernel launch) and, for N > 1, the RCCL gather of
every rank's row bands to rank 0 plus the root-side assembly of the frame.
Inputs (scene, noise buffers, lights) are resident in HBM before timing.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "simple-ray-tracer_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="rubik", choices=("rubik", "spheres", "synthetic"))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--max-depth", type=int, default=5)
    ap.add_argument("--synthetic-tris", type=int, default=10_000_000)
    ap.add_argument("--band-rows", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target length of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def algorithmic_bytes(st: dict) -> int:
    """Bytes one sample_kernel launch must move (SURVEY.md 8d per-unit prices): 32 B per node box test,
    40 B per triangle test, 48 B per mesh-material fetch, 4 B per uniform-noise fetch, 8 B per jitter
    fetch, 32 B per light record, and the 16-B radiance store per sample (the sample buffer that
    accumulate_kernel sums; it replaces the reference's per-frame 32-B accumulation RMW)."""
    return (32 * st["nodes"] + 40 * st["tris"] + 48 * st["mat_reads"] + 4 * st["rng_u"] + 8 * st["rng_sq"]
            + 32 * st["light_reads"] + 16 * st["samples"])


def cpu_baseline(setup, spp_first: int, target_s: float) -> dict:
    """The oracle (scalar C restatement, OpenMP over rows) on this host, on a bounded sample of the workload:
    every 8th row of the frame, full width, consecutive frames of the same progressive sequence."""
    from oracle import pyoracle as O

    s = setup
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    orc = O.Oracle(s.scene, s.lights, s.noise, s.noise_u)
    cam = s.camera
    f = O.Oracle.frame(s.width, s.height, show_model=s.show_model, bvh_count=s.bvh_count, light_count=len(s.lights),
                       max_depth=s.max_depth, origin=cam.position, direction=cam.front, up=cam.up, right=cam.right)
    acc = np.zeros((s.height, s.width, 4), np.float32)
    out = np.zeros((s.height, s.width, 4), np.uint8)
    rows = np.arange(0, s.height, 8, dtype=np.int32)
    # calibrate on one frame, then size the sample to ~target_s
    t0 = time.perf_counter()
    st = orc.render_rows(f, spp_first, 1, acc, out, rows, threads)
    t1 = time.perf_counter()
    frames = max(1, int(target_s / max(t1 - t0, 1e-3)) - 1)
    frames = min(frames, 255)
    t2 = time.perf_counter()
    st2 = orc.render_rows(f, spp_first + 1, frames, acc, out, rows, threads)
    t3 = time.perf_counter()
    rays = st["rays"] + st2["rays"]
    secs = (t1 - t0) + (t3 - t2)
    return {"value": rays / secs / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"oracle on {len(rows)} rows (every 8th) x {s.width} px x {frames + 1} frames of the same "
                      f"workload ({rays} rays, {secs:.1f} s)"}


def load_traffic(workload: str):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary for this workload, if any."""
    p = ROOT / "profiles" / "traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        v = d.get(workload)
        return None if v is None else float(v["hbm_bytes_per_launch"])
    except Exception:
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import srt_amd as S
    from srt_amd import render as R

    W, H, spp = args.width, args.height, args.spp
    if args.scene == "rubik":
        models = [R.rubik_model(ROOT / "tests" / "golden" / "objects")]
        show_model, wl_name = True, f"rubik_{W}x{H}_{spp}spp"
    elif args.scene == "synthetic":
        models = [R.synthetic_model(args.synthetic_tris)]
        show_model, wl_name = True, f"synthetic{args.synthetic_tris}_{W}x{H}_{spp}spp"
    else:
        models, show_model, wl_name = None, False, f"spheres_{W}x{H}_{spp}spp"
    if args.max_depth != 5:
        wl_name += f"_depth{args.max_depth}"
    setup = R.make_setup(W, H, show_model=show_model, models=models, max_depth=args.max_depth)

    dev = torch.device("cuda", local_rank)
    stream = torch.cuda.Stream(device=dev)   # a real (non-null) stream shared by torch and the library
    torch.cuda.set_stream(stream)
    rdr = R.Renderer(setup, device=local_rank, stream=stream.cuda_stream, rank=rank, nranks=world,
                     band_rows=args.band_rows)
    c = rdr.compute
    from srt_amd import parallel as PAR

    rows_pad = PAR.rows_pad(H, args.band_rows, world)
    local_rows = c.local_rows()
    accum_local = torch.zeros((rows_pad, W, 4), dtype=torch.float32, device=dev)
    out_local = torch.zeros((rows_pad, W), dtype=torch.int32, device=dev)
    c.set_image_buffers(accum_local.data_ptr(), out_local.data_ptr())
    if rank == 0 and world > 1:
        full_accum = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
        full_out = torch.empty((H, W), dtype=torch.int32, device=dev)

    # deterministic counting run (untimed): the work every step repeats
    rdr.render(spp, count=True, write_output=True)
    torch.cuda.synchronize()
    st = c.stats()
    counts = torch.tensor([st[k] for k in ("rays", "nodes", "tris", "rng_u", "rng_sq", "light_reads", "mat_reads",
                                           "samples")], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(counts)
    total_rays = float(counts[0].item())
    local_bytes = algorithmic_bytes(st)

    kernel_ms = []

    def step(timed: bool):
        rdr.clear()
        c.render_frames(2, spp, write_output=(world == 1), count=False)
        rdr.accum_frames = spp + 1
        if world > 1:  # the one exchange: every rank's radiance rows to rank 0 (RCCL over xGMI)
            stacked = PAR.gather_bands(accum_local, dst=0)
            if rank == 0:
                c.assemble_bands(stacked.data_ptr(), world, rows_pad, args.band_rows, spp + 1,
                                 full_accum.data_ptr(), full_out.data_ptr())

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
        torch.cuda.synchronize()
        kernel_ms.append(c.last_kernel_ms())  # HIP events around sample_kernel on the launch stream
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed_s = float(elapsed.item())

    if rank == 0:
        ms_per_step = elapsed_s * 1e3 / args.steps
        value = total_rays * args.steps / elapsed_s / 1e6
        k_ms = float(np.mean(kernel_ms))
        achieved = local_bytes / (k_ms * 1e-3) / 1e9
        traffic = load_traffic(wl_name) if world == 1 else None
        line = {
            "metric": "Mrays/s (CheckHit queries: camera + bounce + shadow rays) at the BASELINE frame/spp",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic inputs: glibc-rand noise buffers as the reference generates them; "
                    + ("Rubik.obj (the reference's shipped model scene; the Airplane OBJ is absent from its checkout)"
                       if args.scene == "rubik" else f"{args.scene} scene"),
            "config": {
                "workload": wl_name, "width": W, "height": H, "spp": spp, "max_depth": args.max_depth,
                "scene": args.scene, "lights": int(len(setup.lights)),
                "parallelism": f"row-band tiling x{world} ({args.band_rows}-row bands) + RCCL gather" if world > 1
                else "single GPU",
            },
            "frame_ms": round(ms_per_step / spp, 4),
            "msamples_per_s": round(W * H * spp * args.steps / elapsed_s / 1e6, 3),
            "rays_per_step": int(total_rays),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "kernel": "srt::sample_kernel<false, LDS, BLOCK> (HIP-event time per launch)",
                "kernel_ms": round(k_ms, 3),
                "algorithmic_bytes_per_launch": int(local_bytes),
                "note": "SURVEY 8d bytes (node/triangle/material/noise/light reads) per launch / kernel time. "
                        "The scene is read from its LDS copy and the noise from L2/MALL, so these bytes are not "
                        "HBM traffic (measured HBM bytes: traffic) and frac > 1 means on-chip reuse. The kernel is "
                        "bound by VALU issue under divergence (DESIGN.md section 5).",
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(setup, 2, args.cpu_seconds)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    rdr.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
