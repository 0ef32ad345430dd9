#!/usr/bin/env python3
"""A/B of launch-shape knobs on multi-frame calls (rt_render_frames_device, K views of the view per
call, one call at a time on one stream) in ONE process, interleaved rounds (r05).

Per variant: a fresh scene with the knobs set, 30 warm-up calls (batch order and launch trials
settle), then `calls` timed calls; every frame checked against a single-frame render of the view.
Usage: python tools/ab_multi.py WORKLOAD '[{"knob": v, ...}, ...]' [rounds] [calls] [K]
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

wl_name = sys.argv[1]
variants = json.loads(sys.argv[2])
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 40
K = int(sys.argv[5]) if len(sys.argv) > 5 else 4
wl = bench.WORKLOADS[wl_name]
dev = torch.device("cuda", 0)
d = tempfile.mkdtemp()
path = bench.workload_scene(wl["scene"], d)
p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"],
                   lights=[list(x) for x in wl["lights"]])
cp = p.to_c()
n = wl["width"] * wl["height"] * 3
st = torch.cuda.current_stream(dev)
bufs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(2 * K)]
ref = None
results = {i: [] for i in range(len(variants))}
for rnd in range(rounds):
    for i, v in enumerate(variants):
        with R.Scene.load(path, device=0) as sc:
            for k, val in v.items():
                sc.tune(k, int(val))
            if ref is None:
                sc.render_frame_device(cp, 16, 16, bufs[0].data_ptr(), n, st.cuda_stream)
                torch.cuda.synchronize()
                ref = bufs[0].clone()

            def call(j):
                b = bufs[(j % 2) * K:(j % 2) * K + K]
                sc.render_frames_device([cp] * K, 16, 16, [x.data_ptr() for x in b], n, st.cuda_stream)
            for j in range(30):
                call(j)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for j in range(calls):
                call(j)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / (calls * K) * 1e3
            assert all(torch.equal(b, ref) for b in bufs), f"variant {v}: frame differs"
            tr = sc.trials() if hasattr(sc, "trials") else None
            results[i].append(ms)
            print(f"round {rnd} {json.dumps(v)}: {ms:.4f} ms per frame ({K} per call)"
                  + (f", trials {tr}" if tr is not None else ""), flush=True)
print("summary (median over rounds):")
for i, v in enumerate(variants):
    print(f"  {json.dumps(v)}: {np.median(results[i]):.4f} ms per frame")
