#!/usr/bin/env python3
"""Host-side cost of one rt_render_frames_device call of eight camera-path views (C4), the part of a
timed run's first call the GPU waits for: after a warm-up, per call the host time of the Python
wrapper (ctypes arrays built per call) and of the C entry alone (arrays built beforehand), each
measured with the GPU busy behind earlier calls (no synchronisation inside the timed calls).
Usage: python tools/host_call_probe.py [calls]
"""
import ctypes as C
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
from raytracert_amd import _capi, scenes  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 40
wl = bench.WORKLOADS["c4"]
W, H = wl["width"], wl["height"]
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
views = [R.RenderParams(width=W, height=H, pf=wl["pf"], max_lvl=wl["max_lvl"], lights=[list(x) for x in wl["lights"]],
                        corners=scenes.orbit_corners(W, H, k, 0.25)).to_c() for k in range(8)]
bufs = [torch.zeros(H * W * 3, dtype=torch.uint8, device=dev) for _ in range(8)]
ptrs = [b.data_ptr() for b in bufs]
out = {}
with R.Scene.load(path, device=0) as sc:
    for _ in range(60):
        sc.render_frames_device(views, 16, 16, ptrs, bufs[0].numel(), st.cuda_stream)
    torch.cuda.synchronize(dev)
    # the Python wrapper, as bench.py calls it
    t = []
    for _ in range(calls):
        t0 = time.perf_counter()
        sc.render_frames_device(views, 16, 16, ptrs, bufs[0].numel(), st.cuda_stream)
        t.append(time.perf_counter() - t0)
    torch.cuda.synchronize(dev)
    out["wrapper_us"] = sorted(x * 1e6 for x in t)[len(t) // 2]
    # the C entry alone
    arr = (_capi.RtParams * 8)(*views)
    outs = (C.c_void_p * 8)(*ptrs)
    lib = _capi.lib()
    t = []
    for _ in range(calls):
        t0 = time.perf_counter()
        rc = lib.rt_render_frames_device(sc._h, arr, 8, 16, 16, outs, bufs[0].numel(), C.c_void_p(st.cuda_stream), None)
        t.append(time.perf_counter() - t0)
        assert rc == 0
    torch.cuda.synchronize(dev)
    out["c_entry_us"] = sorted(x * 1e6 for x in t)[len(t) // 2]
    # a call after an idle GPU (what a timed run's first call is): wrapper host time, then the wall
    # clock to its completion
    t, w = [], []
    for _ in range(10):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        sc.render_frames_device(views, 16, 16, ptrs, bufs[0].numel(), st.cuda_stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        t.append((t1 - t0) * 1e6)
        w.append((t2 - t0) * 1e6)
    out["idle_call_host_us"] = sorted(t)[5]
    out["idle_call_wall_us"] = sorted(w)[5]
print(json.dumps(out))
