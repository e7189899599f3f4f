"""Image-space sharding of a frame across GPUs (BASELINE.json configs[3] "C4").

The reference's only parallelism is one task per 8-row chunk
(RT/Extensions/Object+Extension.swift:75-82, 285-376); pixels are independent because
each pixel seeds its own PCG32 (:294).  Across GPUs the same chunks are dealt
round-robin — chunk c -> rank c mod N — which balances sky and terrain rows.  There is
no collective on the render path: each rank renders its chunks from its own full scene
replica into its own buffer; a host-side gather assembles the frame only when a caller
wants the image on one host (outside any timed region).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def chunk_selection(rank: int, world: int) -> Tuple[int, int]:
    """(chunk_first, chunk_step) of `rank`'s share: chunks rank, rank+world, ..."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return rank, world


def rows_of(height: int, first: int, step: int) -> List[Tuple[int, int]]:
    """Row ranges [start, end) of the selected 8-row chunks, in output order."""
    n = (max(1, height) + 7) // 8
    return [(8 * c, min(8 * c + 8, height)) for c in range(first, n, step)]


def assemble(parts: Sequence[Tuple[int, int, np.ndarray]], height: int, width: int, channels: int = 3,
             dtype=np.float64) -> np.ndarray:
    """Scatter each rank's packed rows (first, step, rows[R, W, C]) into one frame."""
    out = np.empty((height, width, channels), dtype=dtype)
    filled = np.zeros(height, dtype=bool)
    for first, step, rows in parts:
        k = 0
        for s, e in rows_of(height, first, step):
            out[s:e] = rows[k:k + (e - s)]
            filled[s:e] = True
            k += e - s
        if k != rows.shape[0]:
            raise ValueError("row count mismatch for shard")
    if not filled.all():
        raise ValueError("missing rows after assembly")
    return out


def render_sharded(renderer, rank: int, world: int, camera_index: int = 0, height: int = None, width: int = None,
                   group=None, dst: int = 0):
    """Render this rank's chunks with `renderer.render_rows(camera_index, first, step)` and gather
    them to rank `dst` (torch.distributed gather_object; gloo or nccl).  Returns the full
    frame on `dst`, None elsewhere."""
    import torch.distributed as dist
    first, step = chunk_selection(rank, world)
    rgb = renderer.render_rows(camera_index, first, step)[0]
    parts = [None] * world if rank == dst else None
    dist.gather_object((first, step, rgb), parts, dst=dst, group=group)
    if rank != dst:
        return None
    return assemble(parts, height, width, rgb.shape[-1], rgb.dtype)
