#!/usr/bin/env python3
"""What rank 0 pays per weak-scaling step at N ranks (r05), measured on one GPU: the render of one
rank's share of N frames (rt_render_tiles_device, frames = N x K, first = 0, stride = N) and the
device un-permute of N x K gathered frames (rt_assemble_tiles_device), each timed with events over
repeated launches; K = steps per call. The gathered buffer is rank 0's shard repeated (the bytes do not
matter for the un-permute's time). Usage: python tools/shard_probe.py [N ...]
"""
import os
import sys
import tempfile
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402
from raytracert_amd import dist as rdist  # noqa: E402

wl = bench.WORKLOADS["c4"]
W, H = wl["width"], wl["height"]
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
p = R.RenderParams(width=W, height=H, pf=wl["pf"], max_lvl=wl["max_lvl"], lights=[list(x) for x in wl["lights"]])
layout = rdist.TileLayout(W, H, 16, 16)
ns = [int(a) for a in sys.argv[1:]] or [2, 8]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    torch.cuda.synchronize(dev)
    return a.elapsed_time(b) / reps


with R.Scene.load(path, device=0) as sc:
    for N in ns:
        for K in (1, 4):
            plan = rdist.ShardPlan(layout, N, frames=N * K)
            shard = torch.zeros(plan.shard_bytes, dtype=torch.uint8, device=dev)
            gathered = shard.repeat(N)
            out = torch.zeros(N * K * H * W * 3, dtype=torch.uint8, device=dev)

            def render():
                sc.render_tiles_device(p, 16, 16, 0, N, shard.data_ptr(), shard.numel(), st.cuda_stream, frames=N * K)

            def assemble():
                R.assemble_tiles_device(0, W, H, 16, 16, N * K, N, gathered.data_ptr(), gathered.numel(), out.data_ptr(),
                                        out.numel(), st.cuda_stream)
            for _ in range(30):
                render()
            torch.cuda.synchronize(dev)
            t_r = timed(render, 20)
            t_a = timed(assemble, 20)
            print(f"N {N} K {K}: render of one rank's share {t_r:.4f} ms ({t_r / K:.4f} per step), un-permute of "
                  f"{N * K} frames {t_a:.4f} ms ({t_a / K:.4f} per step, {2 * N * K * H * W * 3 / t_a / 1e6:.0f} GB/s)",
                  flush=True)
