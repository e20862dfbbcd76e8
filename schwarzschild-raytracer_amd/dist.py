"""Row-band tiling of one frame over the ranks of a node and the gather of the
tiles to rank 0. One process per GPU; torch.distributed with
backend "nccl" is RCCL over xGMI on ROCm ("gloo" for CPU tests).

Partition: the frame's rows are cut into blocks of `block_rows`; block b goes
to rank b % world (block-cyclic). Rows through the photon ring cost ~2x the
edge rows, so contiguous bands are imbalanced (max/mean 1.14 at 8 ranks);
interleaving 8-row blocks keeps every rank within a few % of the mean while
each 8-row block still maps onto whole 8x8 wave tiles.

Exchange: every rank packs its blocks densely into an equal-size tile
(padded to the largest share; sr_render_blocks writes exactly that layout)
and one `gather` brings all tiles to rank 0 into one [world, tile_rows, W, 4]
buffer. Because block b = k*world + rank sits at slot (rank, k), the frame is
that buffer transposed to (k, rank) — a single device copy. With RCCL each
peer's tile travels over its own xGMI link into rank 0.
"""
from __future__ import annotations

import numpy as np


def nblocks(height: int, block_rows: int) -> int:
    return (height + block_rows - 1) // block_rows


def blocks_of(rank: int, world: int, height: int, block_rows: int) -> list[int]:
    return list(range(rank, nblocks(height, block_rows), world))


def rows_of(rank: int, world: int, height: int, block_rows: int) -> list[int]:
    rows = []
    for b in blocks_of(rank, world, height, block_rows):
        rows.extend(range(b * block_rows, min(height, (b + 1) * block_rows)))
    return rows


def tile_rows(world: int, height: int, block_rows: int) -> int:
    """Rows of the equal-size tile every rank contributes to the gather."""
    return ((nblocks(height, block_rows) + world - 1) // world) * block_rows


def assemble(stacked, world: int, height: int, block_rows: int):
    """[world, tile_rows, W, C] gathered tiles (rank order) -> [height, W, C]
    frame. numpy arrays or torch tensors. Batched tiles [world, B, tile_rows,
    W, C] -> [B, height, W, C] frames."""
    if stacked.ndim == 5:
        B = stacked.shape[1]
        if isinstance(stacked, np.ndarray):
            return np.stack([assemble(stacked[:, b], world, height, block_rows) for b in range(B)])
        tr, rest = stacked.shape[2], tuple(stacked.shape[3:])
        per = tr // block_rows
        v = stacked.reshape((world, B, per, block_rows) + rest).permute((1, 2, 0, 3) + tuple(range(4, 4 + len(rest))))
        return v.reshape((B, per * world * block_rows) + rest)[:, :height]
    w, tr = stacked.shape[0], stacked.shape[1]
    assert w == world and tr % block_rows == 0
    rest = tuple(stacked.shape[2:])
    per = tr // block_rows
    v = stacked.reshape((world, per, block_rows) + rest)
    if isinstance(v, np.ndarray):
        v = v.transpose((1, 0, 2) + tuple(range(3, v.ndim)))
        return np.ascontiguousarray(v.reshape((per * world * block_rows,) + rest)[:height])
    v = v.permute((1, 0, 2) + tuple(range(3, v.dim())))
    return v.reshape((per * world * block_rows,) + rest)[:height]


class FrameGather:
    """Preallocated gather of equal-size tiles to rank 0 (collective). A tile
    of [B, tile_rows, W, C] holds B frames (a batched launch); __call__(n)
    gathers the first n of them and returns the [n, H, W, C] frames."""

    def __init__(self, tile, world: int, rank: int, height: int, block_rows: int, group=None):
        self.world, self.rank, self.height, self.block_rows, self.group = world, rank, height, block_rows, group
        self.tile = tile
        self.stacked = None
        self.views = None
        if rank == 0 and world > 1:
            self.stacked = tile.new_empty((world,) + tuple(tile.shape))
            self.views = [self.stacked[i] for i in range(world)]

    def __call__(self, n: int | None = None, assemble_frame: bool = True):
        import torch.distributed as dist

        tile, views, stacked = self.tile, self.views, self.stacked
        if n is not None:  # batched tile: its first n frames
            tile = tile[:n]
            views = None if views is None else [v[:n] for v in views]
            stacked = None if stacked is None else stacked[:, :n]
        if self.world == 1:
            stacked = tile[None]
        else:
            dist.gather(tile, views if self.rank == 0 else None, dst=0, group=self.group)
        if self.rank != 0:
            return None
        if not assemble_frame:
            return stacked
        return assemble(stacked, self.world, self.height, self.block_rows)
