#!/usr/bin/env python3
"""Strong-scaling shares on one GPU (bench.strong_shares) under launch-shape variants.
Usage: python tools/strong_probe.py WORKLOAD [NS] [VARIANT ...]
  NS: comma list of rank counts (default 2,4,8); VARIANT: name:knob=value,knob=value (or 'default').
Prints one JSON line per variant: the frame time t1 (one at a time) and the shares."""
import json
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
ns = tuple(int(x) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else (2, 4, 8)
variants = sys.argv[3:] or ["default"]
W, H = wl["width"], wl["height"]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
st = torch.cuda.current_stream(dev)
path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
flags = R.ALL_FEATURES | (R._capi.STOCHASTIC if wl.get("stochastic") else 0)
p = R.RenderParams(width=W, height=H, pf=wl["pf"], max_lvl=wl["max_lvl"], lights=[list(x) for x in wl["lights"]],
                   flags=flags).to_c()

with R.Scene.load(path, device=0) as sc:
    fb = torch.zeros(H * W * 3, dtype=torch.uint8, device=dev)
    for v in variants:
        name, _, kv = v.partition(":")
        sc.tune("forget_order", 1)
        for item in filter(None, kv.split(",")):
            k, val = item.split("=")
            sc.tune(k, int(val, 0))
        # t1: the whole frame, one at a time (the one-GPU reference point)
        n = 0
        while n < 64 and sc.trials()["choice"] < 0:
            sc.render_frame_device(p, 16, 16, fb.data_ptr(), fb.numel(), st.cuda_stream)
            torch.cuda.synchronize(dev)
            n += 1
        for _ in range(10):
            sc.render_frame_device(p, 16, 16, fb.data_ptr(), fb.numel(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(15):
            t0 = time.perf_counter()
            sc.render_frame_device(p, 16, 16, fb.data_ptr(), fb.numel(), st.cuda_stream)
            torch.cuda.synchronize(dev)
            ts.append((time.perf_counter() - t0) * 1e3)
        t1 = sorted(ts)[len(ts) // 2]
        t0 = time.perf_counter()
        shares = bench.strong_shares(sc, p, W, H, dev, ns=ns)
        el = time.perf_counter() - t0
        brief = {k: {"max_ms": d["max_ms"], "mean_ms": d["mean_ms"], "pipelined_max_ms": d["pipelined_max_ms"],
                     "assemble_ms": d["assemble_ms"], "t1_over_n": round(t1 / int(k[1:]), 4),
                     "max_batch_us": max(r["max_batch_us"] or 0 for r in d["ranks"]),
                     "choices": sorted({(r["choice"], r["steal"], r["dist"]) for r in d["ranks"]})}
                 for k, d in shares.items()}
        print(json.dumps({"workload": sys.argv[1] if len(sys.argv) > 1 else "c4", "variant": v, "t1_ms": round(t1, 4),
                          "probe_s": round(el, 1), "shares": brief}), flush=True)
        print(json.dumps({"variant": v, "detail": shares}), file=sys.stderr, flush=True)
