#!/usr/bin/env python3
"""A new view's first frame (no measured batch order, no launch trial) under cold-launch variants
(r05): per variant a fresh scene with the knobs set, a few warm frames of another view (the GPU and
the library warm), then `reps` cold frames of the C4 view, each after RT_TUNE_FORGET_ORDER,
synchronised and timed on the host. Median per variant, every frame checked against the first.
Usage: python tools/cold_probe.py '[{"cold_estimate": 2}, ...]' [reps]
"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402
from raytracert_amd import scenes  # noqa: E402

variants = json.loads(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
wl = bench.WORKLOADS["c4"]
W, H = wl["width"], wl["height"]
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
mk = lambda c: R.RenderParams(width=W, height=H, pf=wl["pf"], max_lvl=wl["max_lvl"], lights=[list(x) for x in wl["lights"]],
                              corners=c).to_c()
view, other = mk(scenes.orbit_corners(W, H, 0, 0.0)), mk(scenes.orbit_corners(W, H, 40, 0.5))
buf = torch.zeros(H * W * 3, dtype=torch.uint8, device=dev)
ref = None
for rnd in range(2):
    for v in variants:
        with R.Scene.load(path, device=0) as sc:
            for k, x in v.items():
                sc.tune(k, int(x))
            for _ in range(5):
                sc.render_frame_device(other, 16, 16, buf.data_ptr(), buf.numel(), st.cuda_stream)
            torch.cuda.synchronize(dev)
            ts = []
            for _ in range(reps):
                sc.tune("forget_order", 1)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                sc.render_frame_device(view, 16, 16, buf.data_ptr(), buf.numel(), st.cuda_stream)
                torch.cuda.synchronize(dev)
                ts.append((time.perf_counter() - t0) * 1e3)
                if ref is None:
                    ref = buf.clone()
                assert torch.equal(buf, ref), f"variant {v}: frame differs"
            print(f"round {rnd} {json.dumps(v)}: cold frame median {np.median(ts):.4f} ms (min {min(ts):.4f}), "
                  f"longest batch {float(sc.batch_durations().max()):.1f} us", flush=True)
