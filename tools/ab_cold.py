#!/usr/bin/env python3
"""A/B of cold-frame launch shapes (a new view's first frame: no measured batch order) on a bench
workload, in ONE process with interleaved rounds: each variant sets its knobs, drops every measured
order (RT_TUNE_FORGET_ORDER) and times one synchronised rt_render_frame_device with HIP events;
the warm (ordered) frames are timed too (20 back to back). Every variant must give the same bytes.
Usage: python tools/ab_cold.py [workload] [rounds] 'knob=v,knob=v' ..."""
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402

# the library's defaults, restored after each variant (rt_capi.cpp rt_scene)
KNOB_DEFAULTS = {"cold_estimate": 2, "bvh_grid": 16384, "chain_split": 5, "dyn_group": 2, "wave_steal": 2,
                 "pixel_order": 2, "steal_half": 512, "steal_quarter": 0, "split_eighth": 0, "prio_batches": 0,
                 "order_every": 8, "batch_order": 1, "shadow_helpers": 1}
wl_name = sys.argv[1] if len(sys.argv) > 1 else "c4"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
variants = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in v.split(",") if kv) for v in (sys.argv[3:] or [""])]
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
        for _ in range(3):
            sc.render_frame_device(cp, 16, 16, fb.data_ptr(), n, stream.cuda_stream)
        stream.synchronize()
        ref = fb.cpu().numpy()
        defaults = {}
        res = {i: ([], []) for i in range(len(variants))}

        def timed(frames=1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(frames):
                sc.render_frame_device(cp, 16, 16, fb.data_ptr(), n, stream.cuda_stream)
            b.record(stream)
            b.synchronize()
            return a.elapsed_time(b) / frames

        for r in range(rounds):
            for i, v in enumerate(variants):
                for k, val in v.items():
                    sc.tune(k, val)
                sc.tune("forget_order", 1)
                res[i][0].append(timed())
                assert np.array_equal(fb.cpu().numpy(), ref), f"variant {v} changed the image"
                for _ in range(24):   # (the batch order converges, then the launch trials run)
                    sc.render_frame_device(cp, 16, 16, fb.data_ptr(), n, stream.cuda_stream)
                res[i][1].append(timed(20))
                for k in v:   # back to the library defaults for the next variant
                    sc.tune(k, KNOB_DEFAULTS[k])
        for i, v in enumerate(variants):
            c, w = res[i]
            print(f"{wl_name} {v or 'defaults'}: cold median {np.median(c):.4f} ms (min {min(c):.4f}); "
                  f"warm median {np.median(w):.4f} ms")
