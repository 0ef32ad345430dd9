#!/usr/bin/env python3
"""Where a C4 frame's time goes, by feature (r05, diagnostic): 4-frame calls (one chain launch each)
with the reference's features switched off one at a time (rt_params.flags: specular, shadows,
diffuse, ambient) and with max_lvl 0 (no secondary rays), against all on. The differences bound each
feature's share of the launch (the frames differ, so no parity check applies).
Usage: python tools/flags_probe.py [calls]
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
from raytracert_amd import _capi  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 40
wl = bench.WORKLOADS["c4"]
W, H = wl["width"], wl["height"]
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
bufs = [torch.zeros(H * W * 3, dtype=torch.uint8, device=dev) for _ in range(8)]
ALL = _capi.ALL_FEATURES
variants = [("all", ALL, wl["max_lvl"]), ("no specular", ALL & ~_capi.SPECULAR, wl["max_lvl"]),
            ("no shadows", ALL & ~_capi.SHADOWS, wl["max_lvl"]), ("no diffuse", ALL & ~_capi.DIFFUSE, wl["max_lvl"]),
            ("no secondary (max_lvl 0)", ALL, 0), ("no shadows, no secondary", ALL & ~_capi.SHADOWS, 0)]
for rnd in range(2):
    for name, flags, lvl in variants:
        with R.Scene.load(path, device=0) as sc:
            p = R.RenderParams(width=W, height=H, pf=wl["pf"], max_lvl=lvl, lights=[list(x) for x in wl["lights"]],
                               flags=flags).to_c()

            def call(j):
                b = bufs[(j % 2) * 4:(j % 2) * 4 + 4]
                sc.render_frames_device([p] * 4, 16, 16, [x.data_ptr() for x in b], bufs[0].numel(), st.cuda_stream)
            for j in range(30):
                call(j)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for j in range(calls):
                call(j)
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t0) / (4 * calls) * 1e3
            c = sc.render_frame_device(p, 16, 16, bufs[0].data_ptr(), bufs[0].numel(), st.cuda_stream, want_counts=True)
            print(f"round {rnd} {name}: {ms:.4f} ms per frame, rays {[int(x) for x in c]}", flush=True)
