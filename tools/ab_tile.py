#!/usr/bin/env python3
"""A/B of the frame's tile shape (which pixels share a 64-lane wave batch: tile-major samples, so
16x16 tiles give 16x4-pixel batches, 8x8 tiles 8x8-pixel ones) on a bench workload, in ONE
process with interleaved rounds, timing rt_render_frame_device with HIP events on its stream.
Every shape must give the same bytes (pixels are independent). A shape WxH/K also sets
RT_TUNE_PIXEL_ORDER to K (0 row-major, 1 Morton, 2 auto). Usage:
  python tools/ab_tile.py [workload] [rounds] [WxH[/K] ...]"""
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402

wl_name = sys.argv[1] if len(sys.argv) > 1 else "c4"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
def parse(v):
    shape, _, order = v.partition("/")
    w, h = (int(t) for t in shape.split("x"))
    return (w, h, int(order) if order else 2)


shapes = [parse(v) for v in (sys.argv[3:] or ["16x16/0", "16x16/1", "8x8/0"])]
wl = bench.WORKLOADS[wl_name]
with tempfile.TemporaryDirectory() as d:
    path = bench.workload_scene(wl["scene"], d)
    p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"],
                       lights=[list(x) for x in wl["lights"]])
    cp = p.to_c()
    with R.Scene.load(path, device=0) as sc:
        stream = torch.cuda.Stream()
        n = wl["width"] * wl["height"] * 3
        fb = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        ref = None
        res = {s: [] for s in shapes}
        for r in range(rounds):
            for s in shapes:
                sc.tune("pixel_order", s[2])
                for _ in range(8):   # the shape's batch order and steal trials
                    sc.render_frame_device(cp, s[0], s[1], fb.data_ptr(), n, stream.cuda_stream)
                stream.synchronize()
                out = fb.cpu().numpy()
                if ref is None:
                    ref = out
                assert np.array_equal(out, ref), f"tile {s} changed the image"
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                for _ in range(40):
                    sc.render_frame_device(cp, s[0], s[1], fb.data_ptr(), n, stream.cuda_stream)
                b.record(stream)
                b.synchronize()
                res[s].append(a.elapsed_time(b) / 40)
                sc.tune("forget_order", 1)
        for s in shapes:
            v = res[s]
            print(f"{wl_name} tile {s[0]}x{s[1]} pixel_order {s[2]}: median {np.median(v):.4f} ms/frame (min {min(v):.4f}, max {max(v):.4f})")
