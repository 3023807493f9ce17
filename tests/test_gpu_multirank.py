"""bench.py's multi-rank path executed end to end on one GPU.

Each rank is a fresh process running bench.py itself (srt_set_tiling, the fused render, the gather of
every rank's packed band rows to rank 0, srt_assemble_bands on rank 0) with the gloo backend, all ranks
on cuda:0 and the gather staged through the host.  The frame rank 0 assembles must be bit-identical to
a 1-rank render of the same workload.  On a multi-GPU node the same code runs with "nccl" (RCCL) and
one GPU per rank.
"""
import os
import pathlib
import signal
import socket
import subprocess
import sys

import numpy as np
import pytest

from srt_amd import render as R
from conftest import OBJECTS, ROOT, bits_equal

pytestmark = pytest.mark.gpu

W, H, SPP = 96, 61, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reference_frame():
    setup = R.make_setup(W, H, show_model=True, models=[R.rubik_model(OBJECTS)])
    r = R.Renderer(setup)
    try:
        r.render(SPP)
        r.finish()
        return r.accum(), r.output()
    finally:
        r.close()


def _run_bench(tmp_path: pathlib.Path, world: int, band: int):
    port = _free_port()
    dump = tmp_path / f"frame_w{world}_b{band}.npz"
    cmd = [sys.executable, "-X", "faulthandler", str(ROOT / "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
           "--width", str(W), "--height", str(H), "--spp", str(SPP), "--band-rows", str(band),
           "--no-cpu-baseline", "--no-global-leg", "--no-surface-leg", "--no-airplane-leg", "--backend", "gloo", "--same-device", "--dump", str(dump)]
    procs = []
    for rank in range(world):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:  # every rank's Python stacks (faulthandler), then the failure
            for q in procs:
                q.send_signal(signal.SIGABRT)
            tails = []
            for q in procs:
                try:
                    tails.append(q.communicate(timeout=20)[1][-4000:])
                except subprocess.TimeoutExpired:
                    q.kill()
                    tails.append("(no exit after SIGABRT)")
            raise AssertionError("ranks did not finish in 120 s:\n" + "\n----\n".join(tails))
        outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
    line = [l for l in outs[0][1].splitlines() if l.startswith("{")]
    assert line, outs[0][1]
    with np.load(dump) as z:
        return z["accum"], z["out"], line[-1]


@pytest.mark.parametrize("world,band", [(2, 2), (3, 8), (4, 2), (1, 2)])
def test_bench_ranks_assemble_the_one_rank_frame(tmp_path, world, band):
    import json

    acc1, out1 = _reference_frame()
    acc, out, line = _run_bench(tmp_path, world, band)
    assert acc.shape == acc1.shape and out.shape == out1.shape
    assert bits_equal(acc, acc1).all()
    assert (out == out1).all()
    j = json.loads(line)
    assert j["n_gpus"] == world and j["value"] > 0


_RCCL_SCRIPT = r"""
import sys, numpy as np, torch, torch.distributed as dist
sys.path[:0] = sys.argv[2:]
from srt_amd import parallel as PAR
from srt_amd import render as R
from conftest import OBJECTS
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[1], world_size=1, rank=0,
                        device_id=torch.device("cuda", 0))
W, H, SPP, BAND = 64, 40, 2, 2
setup = R.make_setup(W, H, show_model=True, models=[R.rubik_model(OBJECTS)])
r = R.Renderer(setup, rank=0, nranks=1, band_rows=BAND)
rows_pad = PAR.rows_pad(H, BAND, 1)
acc = torch.zeros((rows_pad, W, 4), dtype=torch.float32, device="cuda")
out = torch.zeros((rows_pad, W), dtype=torch.int32, device="cuda")
r.compute.set_image_buffers(acc.data_ptr(), out.data_ptr())
r.render(SPP)
r.finish()
stacked = PAR.gather_bands(acc, dst=0, collective=True)   # dist.gather of device memory over RCCL
full = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
full_out = torch.empty((H, W), dtype=torch.int32, device="cuda")
r.compute.assemble_bands(stacked.data_ptr(), 1, rows_pad, BAND, SPP + 1, full.data_ptr(), full_out.data_ptr())
r.finish()
torch.cuda.synchronize()
r.close()
np.savez("rccl_frame.npz", accum=full.cpu().numpy(),
         out=full_out.cpu().numpy().view(np.uint8).reshape(H, W, 4))
print("OK", dist.get_backend())
dist.destroy_process_group()
"""


def test_rccl_gather_through_torch_distributed(tmp_path):
    """bench.py's exchange over the "nccl" backend (RCCL), which the gloo tests above stage through the
    host: one rank, the collective forced, device memory gathered and assembled; the frame is the oracle's."""
    from conftest import PKG, oracle_render

    script = tmp_path / "rccl_one.py"
    script.write_text(_RCCL_SCRIPT)
    res = subprocess.run([sys.executable, str(script), str(_free_port()), str(PKG), str(ROOT / "tests"), str(ROOT)],
                         capture_output=True, text=True, timeout=120, cwd=tmp_path)
    last = res.stdout.strip().splitlines()[-1] if res.stdout.strip() else ""
    assert res.returncode == 0 and last == "OK nccl", res.stdout[-2000:] + res.stderr[-3000:]
    with np.load(tmp_path / "rccl_frame.npz") as z:
        acc, out = z["accum"], z["out"]
    want = oracle_render(R.make_setup(64, 40, show_model=True, models=[R.rubik_model(OBJECTS)]), 2)
    assert bits_equal(acc, want[0]).all() and (out == want[1]).all()
