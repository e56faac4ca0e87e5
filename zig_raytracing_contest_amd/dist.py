"""Multi-GPU image assembly: interleaved tiles per rank, one gather to rank 0.

SURVEY.md §8e: tiles of the output image shard trivially (the reference
already splits pixels into independent blocks, stage3.zig:228-229); each rank
renders the TILE x TILE tiles (32x32) t with t % world == rank into a packed RGB8 buffer
(zrt_tile_pixels order), then ONE gather moves every rank's packed tiles to
rank 0 (RCCL over xGMI on GPUs: torch.distributed "nccl"; gloo on CPU for the
tests), where they are scattered back into the w x h x 3 image.  No reduction:
pixels are disjoint, so there is no all-reduce.
"""
from __future__ import annotations

import numpy as np

from . import native

# Tile edge of the multi-rank split: 32x32 tiles balance 8 ranks to a max/mean
# per-rank time of 1.008 on cfg3 (64x64: 1.039), strong-scaling efficiency
# 0.934 vs 0.906 predicted from every rank's tile set on one GPU
# (tools/rank_time.py, profiles/r04/r04q_rank_time_tiles.log); the image is
# the same for any tile size.
TILE = 32


def rank_pixels(w: int, h: int, rank: int, world: int, tile: int = TILE) -> np.ndarray:
    return native.tile_pixels(w, h, tile, rank, world)


def max_packed(w: int, h: int, world: int, tile: int = TILE) -> int:
    return max(rank_pixels(w, h, r, world, tile).size for r in range(world))


_IDX = {}


def _indices(w, h, world, tile, device):
    import torch
    key = (w, h, world, tile, str(device))
    if key not in _IDX:
        _IDX[key] = [torch.from_numpy(rank_pixels(w, h, r, world, tile).astype(np.int64)).to(device)
                     for r in range(world)]
    return _IDX[key]


def gather_image(packed, w: int, h: int, rank: int, world: int, dist, tile: int = TILE):
    """packed: 1-D uint8 torch tensor of max_packed(...)*3 bytes on this rank's
    device (only the first n_rank*3 bytes are meaningful).  Returns the
    assembled (h, w, 3) uint8 tensor on rank 0 (same device), None elsewhere;
    the unpermute is one index_copy per rank on the device."""
    import torch
    gl = [torch.empty_like(packed) for _ in range(world)] if rank == 0 else None
    dist.gather(packed, gl, dst=0)
    if rank != 0:
        return None
    img = torch.empty((w * h, 3), dtype=torch.uint8, device=packed.device)
    for r, idx in enumerate(_indices(w, h, world, tile, packed.device)):
        img.index_copy_(0, idx, gl[r][: idx.numel() * 3].view(-1, 3))
    return img.view(h, w, 3)


def render_gathered(context, cam, spp: int, max_bounce: int, rank: int, world: int, dist, dev_buf,
                    stats: bool = False, tile: int = TILE):
    """One frame of bench.py's multi-GPU step: this rank's tiles rendered
    straight into `dev_buf` (a device tensor of max_packed(...)*3 bytes,
    zrt_outputs.device_rgb_packed: no host copy), then gather_image to rank 0.
    Returns (assembled (h, w, 3) tensor on rank 0 / None elsewhere, render
    result dict)."""
    res = context.render(cam, spp, max_bounce, rank=rank, num_ranks=world, tile=tile, stats=stats,
                         device_ptr=dev_buf.data_ptr())
    return gather_image(dev_buf, cam.w, cam.h, rank, world, dist, tile), res
