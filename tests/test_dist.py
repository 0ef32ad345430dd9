"""Multi-rank tile sharding on CPU (gloo, world_size 2 and 3): the ShardPlan partition, the one
gather and the device-side un-permute reassemble every frame exactly. A stub stands in for
rt_render_tiles_device (same output contract: tiles first, first+stride, ... of the frame, each
tile_w*tile_h*3 bytes, pixels outside the frame 0); the GPU test
test_gpu_parity.py::test_sharded_tiles_reassemble_to_full_frame covers the real renderer."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raytracert_amd import dist as rdist


def pattern(w, h):
    y, x = np.mgrid[0:h, 0:w]
    img = np.stack([(x * 7 + y * 13) % 251, (x * 3 + 1) % 253, (y * 5 + 2) % 241], -1)
    return img.astype(np.uint8)


def stub_render(layout, first, stride):
    """What rt_render_tiles_device writes for one frame of the reference pattern."""
    img = pattern(layout.width, layout.height)
    tiles = []
    for t in range(first, layout.n_tiles, stride):
        ty, tx = divmod(t, layout.tiles_x)
        tile = np.zeros((layout.tile_h, layout.tile_w, 3), np.uint8)
        part = img[ty * layout.tile_h:(ty + 1) * layout.tile_h, tx * layout.tile_w:(tx + 1) * layout.tile_w]
        tile[: part.shape[0], : part.shape[1]] = part
        tiles.append(tile)
    return np.stack(tiles) if tiles else np.zeros((0, layout.tile_h, layout.tile_w, 3), np.uint8)


def _worker(rank, world, port, mode, result_path, async_op=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    layout = rdist.TileLayout(100, 70, 16, 16)
    plan = rdist.ShardPlan(layout, world, frames=world if mode == "weak" else 1)
    buf = torch.zeros(plan.shard_bytes, dtype=torch.uint8)
    off = 0
    for (_, first, stride) in plan.calls(rank):   # == one multi-frame call: ids rank, rank+world, ...
        t = stub_render(layout, first, stride).reshape(-1)
        buf[off:off + t.size] = torch.from_numpy(t)
        off += t.size
    assert off == plan.rank_tiles(rank) * layout.tile_bytes
    if async_op:   # bench.py's pipelined form: the gather's work handle is waited on later
        gathered, work = rdist.gather_shards(buf, rank, world, async_op=True)
        work.wait()
    else:
        gathered = rdist.gather_shards(buf, rank, world)
    if rank == 0:
        frames = rdist.assemble_plan_torch(gathered, plan).numpy()
        np.save(result_path, frames, allow_pickle=False)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,mode,async_op", [(2, "weak", False), (2, "strong", False), (3, "weak", False),
                                                 (3, "strong", False), (2, "weak", True), (3, "weak", True)])
def test_gloo_shard_gather_assemble(tmp_path, world, mode, async_op):
    out = str(tmp_path / "frames.npy")
    mp.spawn(_worker, args=(world, _free_port(), mode, out, async_op), nprocs=world, join=True)
    frames = np.load(out, allow_pickle=False)
    expect = pattern(100, 70)
    assert frames.shape == ((world if mode == "weak" else 1), 70, 100, 3)
    for f in frames:
        assert np.array_equal(f, expect)


def test_plan_balances_and_covers():
    layout = rdist.TileLayout(1920, 1080, 16, 16)
    assert layout.n_tiles == 120 * 68
    for world in (1, 2, 4, 8):
        for frames in (1, world):
            plan = rdist.ShardPlan(layout, world, frames)
            per_rank = [sum(plan.tiles_in_call(first) for (_, first, _) in plan.calls(r)) for r in range(world)]
            assert sum(per_rank) == plan.total_tiles
            assert max(per_rank) - min(per_rank) <= 1
            if frames == world:
                assert all(n == layout.n_tiles for n in per_rank)   # weak: one frame of tiles per GPU
            idx = plan.gather_index()
            assert len(np.unique(idx)) == plan.total_tiles


def test_host_assemble_matches_torch():
    layout = rdist.TileLayout(50, 37, 16, 16)
    world = 3
    shards = [stub_render(layout, r, world).reshape(-1) for r in range(world)]
    host = layout.assemble(shards)
    assert np.array_equal(host, pattern(50, 37))
    pad = [np.concatenate([s, np.zeros(layout.shard_bytes(world) - s.size, np.uint8)]) for s in shards]
    g = torch.from_numpy(np.concatenate(pad))
    dev = rdist.assemble_torch(g, layout, world).numpy()
    assert np.array_equal(dev, host)
