"""Multi-GPU host logic on CPU: chunk round-robin + gather with torch.distributed (gloo,
world_size 2).  The CPU oracle stands in for a GPU replica so the test runs here; the
assembled frame must equal a single full render bit for bit (pixels are independent,
Object+Extension.swift:294)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from myraytracer_amd import scenes, shard


class OracleRenderer:
    def __init__(self, sc):
        import oracle
        self.o = oracle.OracleScene(sc)

    def render_rows(self, cam, first, step):
        img, st = self.o.render(cam, first, step, threads=2)
        return img, None, st


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = scenes.scaled(scenes.scene_c2(inline=True), 64, 44)     # 6 chunks, last one partial
    full = shard.render_sharded(OracleRenderer(sc), rank, world, 0, 44, 64)
    if rank == 0:
        np.save(out_path, full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_render_equals_full(tmp_path, world):
    out = str(tmp_path / "full.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    sc = scenes.scaled(scenes.scene_c2(inline=True), 64, 44)
    ref = OracleRenderer(sc).render_rows(0, 0, 1)[0]
    assert np.array_equal(got, ref)


def test_assemble_round_robin_partition():
    H, W = 1080, 4
    frame = np.arange(H * W * 3, dtype=np.float64).reshape(H, W, 3)
    for world in [1, 2, 3, 4, 8]:
        parts = []
        for r in range(world):
            f, s = shard.chunk_selection(r, world)
            rows = np.concatenate([frame[a:b] for a, b in shard.rows_of(H, f, s)])
            parts.append((f, s, rows))
        assert np.array_equal(shard.assemble(parts, H, W), frame)
        # every row exactly once, balanced to within one chunk
        counts = [sum(b - a for a, b in shard.rows_of(H, r, world)) for r in range(world)]
        assert sum(counts) == H and max(counts) - min(counts) <= 8
    with pytest.raises(ValueError):
        shard.assemble(parts[:-1], H, W)
