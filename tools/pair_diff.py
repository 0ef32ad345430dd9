#!/usr/bin/env python3
"""Check (r05): a workload's full frame with shadow helpers on (default) and off must be identical.
Usage: python tools/pair_diff.py c3 [lights]"""
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402

wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
W, H = wl["width"], wl["height"]
path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
p = R.RenderParams(width=W, height=H, pf=wl["pf"], max_lvl=wl["max_lvl"], lights=[list(x) for x in wl["lights"]]).to_c()
out = {}
for name, knobs in (("helpers", {}), ("none", {"shadow_helpers": 0})):
    with R.Scene.load(path, device=0) as sc:
        for k, v in knobs.items():
            sc.tune(k, v)
        fb = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda:0")
        for _ in range(3):
            c = sc.render_frame_device(p, 16, 16, fb.data_ptr(), fb.numel(), torch.cuda.current_stream().cuda_stream, want_counts=True)
        torch.cuda.synchronize()
        out[name] = (fb.view(H, W, 3).cpu().numpy(), [int(x) for x in c])
a, b = out["helpers"][0], out["none"][0]
d = np.argwhere(np.any(a != b, axis=2))
print(sys.argv[1], "counts", out["helpers"][1], out["none"][1], "differing pixels", len(d), d[:5].tolist(), flush=True)
