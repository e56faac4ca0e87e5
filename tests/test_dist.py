"""N>1 path on CPU: world_size-2/3 gloo ranks shard the image into
interleaved tiles and gather packed RGB8 to rank 0 (the same code bench.py
uses with RCCL on GPUs).  Every pixel must arrive exactly once, in place."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, w, h, q):
    import torch
    import torch.distributed as dist

    from zig_raytracing_contest_amd import dist as zdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    px = zdist.rank_pixels(w, h, rank, world)
    buf = torch.zeros(zdist.max_packed(w, h, world) * 3, dtype=torch.uint8)
    # synthetic "render": colour = f(pixel index, rank) so misplacement shows
    vals = np.stack([px % 251, (px // 251) % 253, np.full_like(px, rank)], 1).astype(np.uint8)
    buf[: px.size * 3] = torch.from_numpy(vals.reshape(-1))
    img = zdist.gather_image(buf, w, h, rank, world, dist)
    if rank == 0:
        q.put(img.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h", [(2, 130, 70), (3, 200, 96)])
def test_gather_tiles_gloo(world, w, h):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    pix = np.arange(w * h)
    assert np.array_equal(img[..., 0].reshape(-1), (pix % 251).astype(np.uint8))
    assert np.array_equal(img[..., 1].reshape(-1), ((pix // 251) % 253).astype(np.uint8))
    # tile t (zdist.TILE pixels square) belongs to rank t % world
    from zig_raytracing_contest_amd import dist as zdist
    T = zdist.TILE
    tx = (w + T - 1) // T
    owner = (((pix // w) // T) * tx + (pix % w) // T) % world
    assert np.array_equal(img[..., 2].reshape(-1), owner.astype(np.uint8))
