#!/usr/bin/env python3
"""A/B launch-shape variants on the benchmark frame in ONE process (interleaved rounds), reporting
per-kernel milliseconds from HIP events (cdna_hip_programming.md §5.4 rule 24)."""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import raytracert_amd as R  # noqa: E402
from raytracert_amd import scenes  # noqa: E402
from raytracert_amd._capi import KERNEL_CLOSEST_HIT, KERNEL_SHADOW, KERNEL_SHADE, KERNEL_FRAME, KERNEL_CHAIN  # noqa: E402

variants = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [{}]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
spec = getattr(scenes, sys.argv[3]) if len(sys.argv) > 3 else scenes.C4
obj = scenes.write_sphere_grid(spec, tempfile.mkdtemp(), "ab")
sc = R.Scene.load(obj, device=0)
p = R.RenderParams(width=1920, height=1080, pf=1, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
for k, val in json.loads(os.environ.get("AB_REF", "{}")).items():   # knobs of the reference image
    sc.tune(k, val)
ref, _, _ = sc.render(p)
layout_tiles = ((p.width + 15) // 16) * ((p.height + 15) // 16)
dbuf = torch.zeros(layout_tiles * 16 * 16 * 3, dtype=torch.uint8, device="cuda:0")
cstream = torch.cuda.current_stream()
cp = p.to_c()


def wall_ms():
    """One frame through rt_render_tiles_device on the caller's stream, profiling off."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(cstream)
    sc.render_tiles_device(cp, 16, 16, 0, 1, dbuf.data_ptr(), dbuf.numel(), cstream.cuda_stream)
    b.record(cstream)
    b.synchronize()
    return a.elapsed_time(b)


res = {i: [] for i in range(len(variants))}
work = {}
for r in range(rounds):
    for i, v in enumerate(variants):
        for k, val in v.items():
            sc.tune(k, val)
        wall_ms()
        wall = wall_ms()
        sc.reset_stats()
        sc.set_profiling(True)
        u8, _, _ = sc.render(p)
        sc.set_profiling(False)
        assert np.array_equal(u8, ref), f"variant {v} changed the image"
        q = {name: round(sc.kernel_stats(k)[2] / sc.counts()[1]) for name, k in
             (("ch_queries", KERNEL_CLOSEST_HIT), ("shadow_queries", KERNEL_SHADOW))}
        res[i].append({name: sc.kernel_stats(k)[1] for name, k in
                       (("ch", KERNEL_CLOSEST_HIT), ("shadow", KERNEL_SHADOW), ("shade", KERNEL_SHADE), ("frame", KERNEL_FRAME),
                        ("chain", KERNEL_CHAIN))})
        res[i][-1]["wall"] = wall
        if r == 0:   # work counters slow the kernels: count once, untimed
            sc.reset_stats()
            sc.set_profiling(True, count_work=True)
            sc.render(p)
            sc.set_profiling(False)
            work[i] = {name: sc.work_detail(k) for name, k in (("ch", KERNEL_CLOSEST_HIT), ("shadow", KERNEL_SHADOW))}
            work[i].update(q)
for i, v in enumerate(variants):
    med = {k: float(np.median([x[k] for x in res[i]])) for k in res[i][0]}
    tot = sum(v_ for k_, v_ in med.items() if k_ != "wall")
    print(json.dumps({"variant": v, "median_ms": {k: round(x, 3) for k, x in med.items()}, "kernel_sum_ms": round(tot, 3), "wall_ms": round(med["wall"], 3),
                      "work_tests_visits": work[i]}))
