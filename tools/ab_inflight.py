#!/usr/bin/env python3
"""Frames in flight (RT_TUNE_FRAMES_IN_FLIGHT): F consecutive frames of one view queued on F
alternating streams, each into its own device frame buffer, so a frame's launch can start while the
previous frame's longest batches still run. Times 100 frames back to back (host wall clock between
device syncs) for each F, after a warm-up that lets every pipeline's batch order and trials settle,
and checks every buffer against the F = 1 frame. Usage: python tools/ab_inflight.py [workload] [F ...]"""
import os
import sys
import tempfile
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402

wl_name = sys.argv[1] if len(sys.argv) > 1 else "c4"
fs = [int(x) for x in sys.argv[2:]] or [1, 2, 3]
wl = bench.WORKLOADS[wl_name]
with tempfile.TemporaryDirectory() as d:
    path = bench.workload_scene(wl["scene"], d)
    p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"],
                       lights=[list(x) for x in wl["lights"]])
    cp = p.to_c()
    n = wl["width"] * wl["height"] * 3
    with R.Scene.load(path, device=0) as sc:
        ref = None
        for rnd in range(2):
            for F in fs:
                sc.tune("frames_in_flight", F)
                streams = [torch.cuda.Stream() for _ in range(F)]
                bufs = [torch.zeros(n, dtype=torch.uint8, device="cuda:0") for _ in range(F)]
                for i in range(40 * F):
                    k = i % F
                    sc.render_frame_device(cp, 16, 16, bufs[k].data_ptr(), n, streams[k].cuda_stream)
                torch.cuda.synchronize()
                if ref is None:
                    ref = bufs[0].cpu()
                steps = 100
                t0 = time.perf_counter()
                for i in range(steps):
                    k = i % F
                    sc.render_frame_device(cp, 16, 16, bufs[k].data_ptr(), n, streams[k].cuda_stream)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / steps * 1e3
                ok = all(torch.equal(b.cpu(), ref) for b in bufs)
                print(f"{wl_name} round {rnd} frames_in_flight {F}: {ms:.4f} ms/frame, frames equal: {ok}", flush=True)
