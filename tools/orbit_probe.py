#!/usr/bin/env python3
"""Where a moving view's frame loses against a static one (r05): C4 orbit views one at a time,
(a) as the bench's orbit leg renders them (each view once: its order comes from the previous view,
dilated, RT_TUNE_MOTION_ORDER), (b) each view rendered twice and the second timed (its order was
measured on that very view: the best a predicted order can do), (c) the static view. Per mode the
mean frame time and the mean longest batch (rt_batch_durations) over the timed views.
Usage: python tools/orbit_probe.py [step_deg] [views] [motion_order ...]
"""
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

step = float(sys.argv[1]) if len(sys.argv) > 1 else 0.25
nv = int(sys.argv[2]) if len(sys.argv) > 2 else 60
orders = [int(x) for x in sys.argv[3:]] or [1]
wl = bench.WORKLOADS["c4"]
W, H = wl["width"], wl["height"]
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
mk = lambda c: R.RenderParams(width=W, height=H, pf=wl["pf"], max_lvl=wl["max_lvl"], lights=[list(x) for x in wl["lights"]],
                              corners=c).to_c()
views = [mk(scenes.orbit_corners(W, H, k + 1, step)) for k in range(2 * nv + 40)]
static = mk(scenes.orbit_corners(W, H, 0, 0.0))
buf = torch.zeros(H * W * 3, dtype=torch.uint8, device=dev)


def one(sc, p):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    sc.render_frame_device(p, 16, 16, buf.data_ptr(), buf.numel(), st.cuda_stream)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) * 1e3, float(sc.batch_durations().max())


for mo in orders:
    with R.Scene.load(path, device=0) as sc:
        sc.tune("motion_order", mo)
        for k in range(40):   # warm-up: trials decided, order settled on the moving view
            one(sc, views[k])
        a = [one(sc, views[40 + k]) for k in range(nv)]
        b = []
        for k in range(nv):
            one(sc, views[40 + nv + k])
            b.append(one(sc, views[40 + nv + k]))
        for _ in range(30):
            one(sc, static)
        c = [one(sc, static) for _ in range(nv)]
        for name, r in (("moving, each view once", a), ("moving, second render of each view", b), ("static view", c)):
            r = np.array(r)
            print(f"motion_order {mo} {name}: {r[:, 0].mean():.4f} ms per frame (median {np.median(r[:, 0]):.4f}), "
                  f"longest batch {r[:, 1].mean():.1f} us", flush=True)
