#!/usr/bin/env python3
"""One feature variant of the C4 frame as four-frame calls (the headline's chain launch), for the
per-phase VALU breakdown: run once per variant under rocprofv3 --pmc and
subtract (tools/phase_summary.py). Variants switch the reference's features off (rt_params.flags)
or stop the chain at the primary hit (max_lvl 0); the frames differ, so no parity applies here.
Usage: python tools/phase_probe.py VARIANT [calls]
  VARIANT: all | no_specular | no_shadows | no_secondary | no_shadows_no_secondary | no_diffuse
"""
import os
import sys
import tempfile
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402
from raytracert_amd import _capi  # noqa: E402

ALL = _capi.ALL_FEATURES
VARIANTS = {"all": (ALL, None), "no_specular": (ALL & ~_capi.SPECULAR, None), "no_shadows": (ALL & ~_capi.SHADOWS, None),
            "no_secondary": (ALL, 0), "no_shadows_no_secondary": (ALL & ~_capi.SHADOWS, 0),
            "no_diffuse": (ALL & ~_capi.DIFFUSE, None)}
name = sys.argv[1]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
flags, lvl = VARIANTS[name]
wl = bench.WORKLOADS["c4"]
W, H = wl["width"], wl["height"]
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
bufs = [torch.zeros(H * W * 3, dtype=torch.uint8, device=dev) for _ in range(8)]
with R.Scene.load(path, device=0) as sc:
    p = R.RenderParams(width=W, height=H, pf=wl["pf"], max_lvl=wl["max_lvl"] if lvl is None else lvl,
                       lights=[list(x) for x in wl["lights"]], flags=flags).to_c()

    def call(j):
        b = bufs[(j % 2) * 4:(j % 2) * 4 + 4]
        sc.render_frames_device([p] * 4, 16, 16, [x.data_ptr() for x in b], bufs[0].numel(), st.cuda_stream)
    n = 0
    while n < 64 and sc.trials()["choice"] < 0:
        call(n)
        torch.cuda.synchronize(dev)
        n += 1
    for j in range(10):
        call(j)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for j in range(calls):
        call(j)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / (4 * calls) * 1e3
    c = sc.render_frame_device(p, 16, 16, bufs[0].data_ptr(), bufs[0].numel(), st.cuda_stream, want_counts=True)
    print(f"{name}: {ms:.4f} ms per frame, calibration {n}, rays {[int(x) for x in c]}", flush=True)
