"""Screen-tile sharding of a frame across ranks (one process per GPU) and the gather to rank 0.

The frame is cut into T x T tiles in raster order; rank r traces tiles r, r + world, r + 2*world, ... into one
contiguous tile-major buffer (VHX_LAYOUT_TILES: the j-th tile of the rank at [j*T*T, (j+1)*T*T), row-major inside,
zeros past the frame edge). Rank 0 gathers the buffers (RCCL over xGMI with the nccl backend; gloo on CPU) and
scatters them into the framebuffer (vhx_untile_rgba on the GPU; untile_numpy is the host restatement used by tests).
"""
import numpy as np


def tile_grid(width, height, T):
    return (width + T - 1) // T, (height + T - 1) // T


def tiles_per_rank(width, height, T, world):
    tx, ty = tile_grid(width, height, T)
    return (tx * ty + world - 1) // world


def rank_tiles(width, height, T, rank, world):
    tx, ty = tile_grid(width, height, T)
    return list(range(rank, tx * ty, world))


def tile_rect(tile, width, height, T):
    tx, _ = tile_grid(width, height, T)
    x0, y0 = (tile % tx) * T, (tile // tx) * T
    return x0, y0, min(T, width - x0), min(T, height - y0)


def rank_rays(width, height, T, rank, world):
    return sum(w * h for _, _, w, h in (tile_rect(t, width, height, T) for t in rank_tiles(width, height, T, rank, world)))


def untile_numpy(gathered, ranks, per_rank, T, width, height):
    """Host restatement of k_untile_rgba: gathered = concatenation over ranks of per_rank*T*T pixels."""
    fb = np.zeros(width * height, gathered.dtype)
    for r in range(ranks):
        for j, tile in enumerate(range(r, tile_grid(width, height, T)[0] * tile_grid(width, height, T)[1], ranks)):
            x0, y0, w, h = tile_rect(tile, width, height, T)
            blk = gathered[(r * per_rank + j) * T * T:(r * per_rank + j + 1) * T * T].reshape(T, T)
            fb.reshape(height, width)[y0:y0 + h, x0:x0 + w] = blk[:h, :w]
    return fb


def gather_to_root(local, world, rank, dist):
    """torch.distributed.gather of equally sized tile buffers to rank 0; returns the concatenation on rank 0."""
    import torch
    if world == 1:
        return local
    bufs = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
    dist.gather(local, bufs, dst=0)
    return torch.cat(bufs) if rank == 0 else None
