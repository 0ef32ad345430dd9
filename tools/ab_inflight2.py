#!/usr/bin/env python3
"""Frames in flight the way bench.py times them: load, calibrate pipeline 0 one synchronised frame at
a time until its launch trials are decided, set F, W x F warm-up frames, K timed frames on F
alternating streams; then the same K frames one in flight. Variants by extra knobs (KNOB=VALUE,
comma-separated) per argument. Usage: python tools/ab_inflight2.py WORKLOAD K W "knobs" ["knobs" ...]"""
import os
import sys
import tempfile
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402

wl_name, K, W = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
variants = sys.argv[4:] or [""]
wl = bench.WORKLOADS[wl_name]
dev = torch.device("cuda", 0)
with tempfile.TemporaryDirectory() as d:
    path = bench.workload_scene(wl["scene"], d)
    p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"],
                       lights=[list(x) for x in wl["lights"]])
    cp = p.to_c()
    n = wl["width"] * wl["height"] * 3
    for rnd in range(2):
        for v in variants:
            with R.Scene.load(path, device=0) as sc:
                prio, FF = False, 2
                for kv in filter(None, v.split(",")):
                    k, val = kv.split("=")
                    if k == "prio":   # frames in flight on a high- and a low-priority stream
                        prio = bool(int(val))
                        continue
                    if k == "F":      # frames in flight of the in-flight loop (default 2)
                        FF = int(val)
                        continue
                    sc.tune(k, int(val))
                main = torch.cuda.current_stream(dev)
                if prio:
                    lo, hi = torch.cuda.Stream.priority_range()
                    streams = [torch.cuda.Stream(dev, priority=hi), torch.cuda.Stream(dev, priority=lo)]
                    main = streams[0]
                else:
                    streams = [main] + [torch.cuda.Stream(dev) for _ in range(FF - 1)]
                bufs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(max(2, FF))]
                calib = 0
                while calib < 64 and sc.trials()["choice"] < 0:
                    sc.render_frame_device(cp, 16, 16, bufs[0].data_ptr(), n, main.cuda_stream)
                    torch.cuda.synchronize()
                    calib += 1
                ref = bufs[0].clone()
                res = []
                for F in (FF, 1):
                    sc.tune("frames_in_flight", F)
                    for i in range(W * F):
                        sc.render_frame_device(cp, 16, 16, bufs[i % len(bufs)].data_ptr(), n, streams[i % F].cuda_stream)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(K):
                        sc.render_frame_device(cp, 16, 16, bufs[i % len(bufs)].data_ptr(), n, streams[i % F].cuda_stream)
                    torch.cuda.synchronize()
                    res.append((time.perf_counter() - t0) / K * 1e3)
                    assert all(torch.equal(b, ref) for b in bufs)
                print(f"{wl_name} round {rnd} [{v or 'default'}] calib {calib}: {FF} in flight {res[0]:.4f} ms, "
                      f"1 in flight {res[1]:.4f} ms, trials {sc.trials()}", flush=True)
