#!/usr/bin/env python3
"""A/B of launch-shape knobs on one workload's frame in ONE process, interleaved rounds (r05).

Per variant: a fresh scene, the knobs set (plus fixed ones that keep the launch trials out: wave_steal
0, chain_split 0 unless given), 24 warm-up frames (the batch order converges), then K frames one in
flight (back to back on one stream) and K frames two in flight (two torch streams), every
frame checked against the reference frame (the same knobs' first frame with all tiers off); the
longest wave batch of the last launch (rt_batch_durations) is the critical path.
Usage: python tools/ab_frame.py WORKLOAD '[{"knob": v, ...}, ...]' [rounds] [K]
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
K = int(sys.argv[4]) if len(sys.argv) > 4 else 40
wl = bench.WORKLOADS[wl_name]
dev = torch.device("cuda", 0)
d = tempfile.mkdtemp()
path = bench.workload_scene(wl["scene"], d)
p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"],
                   lights=[list(x) for x in wl["lights"]])
cp = p.to_c()
n = wl["width"] * wl["height"] * 3
main = torch.cuda.current_stream(dev)
side = torch.cuda.Stream(dev)
bufs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(2)]
ref = None
results = {i: [] for i in range(len(variants))}
for rnd in range(rounds):
    for i, v in enumerate(variants):
        with R.Scene.load(path, device=0) as sc:
            knobs = {"wave_steal": 0, "chain_split": 0, "shadow_helpers": 1, "steal_quarter": 0}
            knobs.update(v)
            for k, val in knobs.items():
                sc.tune(k, int(val))
            if ref is None:
                sc.render_frame_device(cp, 16, 16, bufs[0].data_ptr(), n, main.cuda_stream)
                torch.cuda.synchronize()
                ref = bufs[0].clone()
            for _ in range(24):
                sc.render_frame_device(cp, 16, 16, bufs[0].data_ptr(), n, main.cuda_stream)
                torch.cuda.synchronize()
            out = {}
            for F in (1, 2):
                sc.tune("frames_in_flight", F)
                streams = [main, side][:F]
                for j in range(4 * F):
                    sc.render_frame_device(cp, 16, 16, bufs[j % 2].data_ptr(), n, streams[j % F].cuda_stream)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for j in range(K):
                    sc.render_frame_device(cp, 16, 16, bufs[j % 2].data_ptr(), n, streams[j % F].cuda_stream)
                torch.cuda.synchronize()
                out[F] = (time.perf_counter() - t0) / K * 1e3
                assert all(torch.equal(b, ref) for b in bufs), f"variant {v}: frame differs"
            sc.tune("frames_in_flight", 1)
            sc.render_frame_device(cp, 16, 16, bufs[0].data_ptr(), n, main.cuda_stream)
            torch.cuda.synchronize()
            bd = sc.batch_durations()
            results[i].append((out[1], out[2], float(bd.max())))
            print(f"round {rnd} {json.dumps(v)}: 1 in flight {out[1]:.4f} ms, 2 in flight {out[2]:.4f} ms, "
                  f"batch max {bd.max():.1f} us, p99 {np.percentile(bd, 99):.1f}", flush=True)
print("summary (median over rounds):")
for i, v in enumerate(variants):
    a = np.array(results[i])
    print(f"  {json.dumps(v)}: 1 in flight {np.median(a[:, 0]):.4f} ms, 2 in flight {np.median(a[:, 1]):.4f} ms, "
          f"batch max {np.median(a[:, 2]):.1f} us")
