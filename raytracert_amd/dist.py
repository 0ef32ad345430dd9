"""Screen-tile sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The frame loop of the reference (CG_Project/main.cpp:369-395) has no cross-pixel state, so the
image is cut into tile_w x tile_h tiles numbered row-major; tile t goes to rank t mod N
(interleaved, which balances the uneven per-region cost: hits cluster where the model is).
Each rank renders its tiles with rt_render_tiles_device into a device buffer, quantised to
uint8 before any exchange (main.cpp:117 is per pixel, so 1-GPU and N-GPU bytes are identical),
and rank 0 collects the shards with ONE gather of equal-sized padded buffers, then un-permutes
the tiles on the device. No other collective touches the data path.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class TileLayout:
    width: int
    height: int
    tile_w: int = 16
    tile_h: int = 16

    @property
    def tiles_x(self) -> int:
        return (self.width + self.tile_w - 1) // self.tile_w

    @property
    def tiles_y(self) -> int:
        return (self.height + self.tile_h - 1) // self.tile_h

    @property
    def n_tiles(self) -> int:
        return self.tiles_x * self.tiles_y

    @property
    def tile_bytes(self) -> int:
        return self.tile_w * self.tile_h * 3

    def tiles_of(self, rank: int, world: int) -> int:
        """Tiles t = rank, rank + world, ... below n_tiles."""
        return (self.n_tiles - rank + world - 1) // world if rank < self.n_tiles else 0

    def max_tiles(self, world: int) -> int:
        return (self.n_tiles + world - 1) // world

    def shard_bytes(self, world: int) -> int:
        """Equal-size shard buffer (padded) so one gather of fixed counts suffices."""
        return self.max_tiles(world) * self.tile_bytes

    def tile_ids(self, world: int) -> np.ndarray:
        """[world, max_tiles] tile id held in each shard slot (-1 = padding)."""
        m = self.max_tiles(world)
        ids = np.arange(world)[:, None] + world * np.arange(m)[None, :]
        ids[ids >= self.n_tiles] = -1
        return ids

    def assemble(self, shards) -> np.ndarray:
        """Host-side un-permute: list of per-rank uint8 shard buffers -> H x W x 3 frame."""
        world = len(shards)
        ids = self.tile_ids(world)
        grid = np.zeros((self.tiles_y * self.tile_h, self.tiles_x * self.tile_w, 3), np.uint8)
        for r, buf in enumerate(shards):
            tiles = np.asarray(buf, np.uint8).reshape(-1, self.tile_h, self.tile_w, 3)
            for k, tid in enumerate(ids[r]):
                if tid < 0 or k >= len(tiles):
                    continue
                ty, tx = divmod(int(tid), self.tiles_x)
                grid[ty * self.tile_h:(ty + 1) * self.tile_h, tx * self.tile_w:(tx + 1) * self.tile_w] = tiles[k]
        return grid[: self.height, : self.width]

    def gather_index(self, world: int):
        """Flat index that maps the gathered [world * max_tiles] tiles onto the padded tile grid
        (row-major tile order): frame_tiles = gathered[index]."""
        ids = self.tile_ids(world).reshape(-1)
        index = np.zeros(self.n_tiles, np.int64)
        valid = ids >= 0
        index[ids[valid]] = np.nonzero(valid)[0]
        return index


def assemble_torch(gathered, layout: TileLayout, world: int, index=None):
    """Device-side un-permute of the gathered shards (torch tensor of world*shard_bytes uint8)
    into an H x W x 3 uint8 frame on the same device."""
    import torch
    tw, th = layout.tile_w, layout.tile_h
    tiles = gathered.view(world * layout.max_tiles(world), th, tw, 3)
    if index is None:
        index = torch.as_tensor(layout.gather_index(world), device=gathered.device)
    grid = tiles.index_select(0, index).view(layout.tiles_y, layout.tiles_x, th, tw, 3)
    frame = grid.permute(0, 2, 1, 3, 4).reshape(layout.tiles_y * th, layout.tiles_x * tw, 3)
    return frame[: layout.height, : layout.width]


def gather_shards(buf, rank: int, world: int, group=None, async_op: bool = False):
    """One collective: gather every rank's equal-sized shard buffer to rank 0. Returns the
    concatenated tensor on rank 0 (None elsewhere); world == 1 returns buf itself. With async_op
    it returns (tensor, work): the gather runs on the collective's own stream and work.wait()
    orders the caller's stream after it, so the next shard can render meanwhile (into another
    buffer)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return (buf, None) if async_op else buf
    out = torch.empty(world * buf.numel(), dtype=buf.dtype, device=buf.device) if rank == 0 else None
    work = dist.gather(buf, list(out.chunk(world)) if rank == 0 else None, dst=0, group=group, async_op=async_op)
    return (out, work) if async_op else out


def render_frame_sharded(render_shard, layout: TileLayout, rank: int, world: int, buf, group=None, index=None):
    """render_shard(buf, first, stride) fills `buf` with this rank's tiles (rank, rank+world,...).
    Returns the assembled frame tensor on rank 0, None on the others."""
    render_shard(buf, rank, world)
    gathered = gather_shards(buf, rank, world, group)
    if rank != 0:
        return None
    return assemble_torch(gathered, layout, world, index)


@dataclass(frozen=True)
class ShardPlan:
    """Tiles of a batch of `frames` frames (identical views), global tile id g = f * T + t,
    interleaved over `world` ranks: rank g % world holds g in slot g // world.

    frames == 1 splits one frame N ways (strong scaling of a frame); frames == world gives every
    rank exactly one frame's worth of tiles (weak scaling: fixed work per GPU)."""
    layout: TileLayout
    world: int
    frames: int = 1

    @property
    def total_tiles(self) -> int:
        return self.frames * self.layout.n_tiles

    @property
    def slots(self) -> int:
        return (self.total_tiles + self.world - 1) // self.world

    @property
    def shard_bytes(self) -> int:
        return self.slots * self.layout.tile_bytes

    def calls(self, rank: int):
        """(frame, first, stride) for each rt_render_tiles_device call of `rank`, in slot order."""
        T = self.layout.n_tiles
        out = []
        for f in range(self.frames):
            first = (rank - f * T) % self.world
            if first < T:
                out.append((f, first, self.world))
        return out

    def tiles_in_call(self, first: int) -> int:
        T = self.layout.n_tiles
        return (T - first + self.world - 1) // self.world if first < T else 0

    def rank_tiles(self, rank: int) -> int:
        """Tiles rank holds: ids rank, rank + world, ... below frames * T (one rt_render_tiles_device
        call with frames=self.frames, first=rank, stride=world)."""
        return (self.total_tiles - rank + self.world - 1) // self.world if rank < self.total_tiles else 0

    def gather_index(self):
        """index[g] = position of global tile g in the gathered [world * slots] tile array."""
        g = np.arange(self.total_tiles, dtype=np.int64)
        return (g % self.world) * self.slots + g // self.world


def assemble_plan_torch(gathered, plan: ShardPlan, index=None):
    """Device-side un-permute of gathered shards into [frames, H, W, 3] uint8."""
    import torch
    L = plan.layout
    tiles = gathered.view(plan.world * plan.slots, L.tile_h, L.tile_w, 3)
    if index is None:
        index = torch.as_tensor(plan.gather_index(), device=gathered.device)
    grid = tiles.index_select(0, index).view(plan.frames, L.tiles_y, L.tiles_x, L.tile_h, L.tile_w, 3)
    frames = grid.permute(0, 1, 3, 2, 4, 5).reshape(plan.frames, L.tiles_y * L.tile_h, L.tiles_x * L.tile_w, 3)
    return frames[:, : L.height, : L.width]
