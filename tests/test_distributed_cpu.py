"""Multi-rank frame tiling on CPU: world_size 2 over gloo, the same band layout and gather the
GPU bench uses (srt_amd.parallel), each rank rendering its bands with the oracle; the root's
assembled frame must be bit-identical to a single-rank render."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from srt_amd import parallel as PAR


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup():
    import srt_amd as S
    from srt_amd import render as R
    from conftest import OBJECTS

    return R.make_setup(40, 37, show_model=True, models=[S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")])


def _worker(rank, world, port, band_rows, q):

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from conftest import oracle_render

    setup = _setup()
    H, W = setup.height, setup.width
    rows = PAR.local_global_rows(H, band_rows, world, rank)
    acc, _, _ = oracle_render(setup, 2, rows=rows.astype(np.int32), threads=1)
    local = np.zeros((PAR.rows_pad(H, band_rows, world), W, 4), np.float32)
    local[:len(rows)] = acc[rows]
    stacked = PAR.gather_bands(torch.from_numpy(local))
    if rank == 0:
        q.put(PAR.assemble_host(stacked.numpy(), H, band_rows))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("band_rows", [8, 16])
def test_two_rank_gloo_tiling_is_bit_identical(band_rows):
    from conftest import oracle_render, bits_equal

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, band_rows, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full, _, _ = oracle_render(_setup(), 2)
    assert bits_equal(frame, full).all()


def test_band_layout_covers_every_row_once():
    for H, band, world in ((1080, 16, 8), (1080, 16, 3), (37, 8, 2), (4096, 16, 8), (7, 16, 4)):
        rows = np.concatenate([PAR.local_global_rows(H, band, world, r) for r in range(world)])
        assert sorted(rows.tolist()) == list(range(H))
        for r in range(world):
            assert len(PAR.local_global_rows(H, band, world, r)) <= PAR.rows_pad(H, band, world)
