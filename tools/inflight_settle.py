#!/usr/bin/env python3
"""How frames in flight settle after the one-in-flight calibration: per 5-frame window of 80 frames
on 2 alternating streams (synchronised at window ends), the ms per frame; and each pipeline's
trial state (rt_scene_trials reports pipeline 0). Usage: tools/inflight_settle.py [workload] [knob=v,...]"""
import os
import sys
import tempfile
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402

wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
dev = torch.device("cuda", 0)
with tempfile.TemporaryDirectory() as d:
    path = bench.workload_scene(wl["scene"], d)
    p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"],
                       lights=[list(x) for x in wl["lights"]])
    cp = p.to_c()
    n = wl["width"] * wl["height"] * 3
    with R.Scene.load(path, device=0) as sc:
        knobs = sys.argv[2] if len(sys.argv) > 2 else ""
        for kv in filter(None, knobs.split(",")):
            k, v = kv.split("=")
            sc.tune(k, int(v))
        main = torch.cuda.current_stream(dev)
        streams = [main, torch.cuda.Stream(dev)]
        bufs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(2)]
        calib = 0
        while calib < 64 and sc.trials()["choice"] < 0:
            sc.render_frame_device(cp, 16, 16, bufs[0].data_ptr(), n, main.cuda_stream)
            torch.cuda.synchronize()
            calib += 1
        pre = int(os.environ.get("SETTLE_PRE", "0"))   # back-to-back one-in-flight frames first (GPU kept busy)
        for i in range(pre):
            sc.render_frame_device(cp, 16, 16, bufs[0].data_ptr(), n, main.cuda_stream)
        torch.cuda.synchronize()
        F = int(os.environ.get("SETTLE_F", "2"))
        one_stream = os.environ.get("SETTLE_ONE_STREAM") == "1"   # frames alternate pipelines on one stream
        if one_stream:
            streams = [main, main]
        sc.tune("frames_in_flight", F)
        win = []
        if os.environ.get("SETTLE_TRACE") == "1":   # the first 8 calls one by one: host time of the call, then of the sync
            tr = []
            for k in range(8):
                t0 = time.perf_counter()
                sc.render_frame_device(cp, 16, 16, bufs[k % 2].data_ptr(), n, streams[k % 2].cuda_stream)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                tr.append((round((t1 - t0) * 1e3, 3), round((time.perf_counter() - t1) * 1e3, 3)))
            print("first calls (host ms, sync ms)", tr, flush=True)
            for k in range(int(os.environ.get("SETTLE_BUSY", "0"))):   # then back-to-back frames (GPU busy)
                sc.render_frame_device(cp, 16, 16, bufs[k % 2].data_ptr(), n, streams[k % 2].cuda_stream)
            torch.cuda.synchronize()
            time.sleep(float(os.environ.get("SETTLE_SLEEP_MS", "0")) / 1e3)   # an idle GPU before the windows
        for w in range(16):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(5):
                k = 5 * w + i
                sc.render_frame_device(cp, 16, 16, bufs[k % 2].data_ptr(), n, streams[k % 2].cuda_stream)
            torch.cuda.synchronize()
            win.append(round((time.perf_counter() - t0) / 5 * 1e3, 4))
        print(knobs or "default", "F", F, "one_stream", one_stream, "pre", pre, "calib", calib, "windows ms/frame", win, "trials", sc.trials(), flush=True)
