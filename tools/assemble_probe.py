#!/usr/bin/env python3
"""rt_assemble_tiles_device alone (the N > 1 step's un-permute on rank 0): HIP-event time per call and
per frame for C4-sized frames (1920x1080, 16x16 tiles) at N ranks and F frames per gather, random shard
bytes, 30 calls after 5 warm-up calls. Usage: python tools/assemble_probe.py [label]
"""
import json
import sys

import torch

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracert_amd as R  # noqa: E402

W, H, TILE = 1920, 1080, 16
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
T = (W // TILE) * ((H + TILE - 1) // TILE)
res = {"label": sys.argv[1] if len(sys.argv) > 1 else ""}
for n in (2, 8):
    for f in (1, 8, 40):
        slots = (f * T + n - 1) // n
        g = torch.randint(0, 256, (n * slots * TILE * TILE * 3,), dtype=torch.uint8, device=dev)
        out = torch.empty(f * H * W * 3, dtype=torch.uint8, device=dev)
        call = lambda: R.assemble_tiles_device(0, W, H, TILE, TILE, f, n, g.data_ptr(), g.numel(), out.data_ptr(), out.numel(),
                                               st.cuda_stream)
        for _ in range(5):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(30):
            call()
        e1.record(st)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / 30
        res[f"n{n}_f{f}"] = {"ms_per_call": round(ms, 4), "us_per_frame": round(ms * 1e3 / f, 2),
                             "TBps": round(2 * f * W * H * 3 / (ms * 1e-3) / 1e12, 2)}
print(json.dumps(res))
