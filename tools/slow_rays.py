#!/usr/bin/env python3
"""Where a frame's slowest chain-launch waves come from (diagnostic -DRT_WAVE_TIMES build via
RTAMD_LIB): renders the workload with the batch order off (wave w = batch w = 64 consecutive
samples of the tile-major queue), maps the slowest waves to screen tiles, then re-traces every
primary ray of the slowest tile one at a time through rt_intersect_mesh in counting mode (and its
shadow ray toward light 0 from the hit point + 0.1, raytracing.cpp:248) and prints the rays with
the most BVH node visits and triangle tests.

    WORKLOAD=c2 RTAMD_LIB=raytracert_amd/ab/lib_wt.so python tools/slow_rays.py
"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402
from raytracert_amd._capi import KERNEL_CLOSEST_HIT  # noqa: E402

wl = bench.WORKLOADS[os.environ.get("WORKLOAD", "c2")]
obj = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
sc = R.Scene.load(obj, device=0)
sc.tune("pipes", 1)
sc.tune("batch_order", 0)
W, H = wl["width"], wl["height"]
p = R.RenderParams(width=W, height=H, pf=1, max_lvl=wl["max_lvl"], lights=wl["lights"])
sc.render(p)
sc.reset_stats()
sc.set_profiling(True, count_work=True)
sc.render(p)
sc.set_profiling(False)
d = sc.diag_read(0, 3 * 43690).reshape(-1, 3).astype(np.int64)
d = d[d[:, 1] > 0]
life = (d[:, 1] - d[:, 0]) * 0.01
tiles_x = (W + 15) // 16
order = np.argsort(-life)
slow = [(int(i) * 64 // 256 % tiles_x, int(i) * 64 // 256 // tiles_x, round(float(life[i]), 1)) for i in order[:12]]
print(json.dumps({"waves": len(d), "median_life_us": round(float(np.median(life)), 1), "slowest_tile_xy_us": slow}))
print(json.dumps({"bvh": sc.bvh_info(), "closest_hit_work": sc.work_detail(KERNEL_CLOSEST_HIT)}))

# every primary ray of the slowest tile (main.cpp:380-386 corner blend, pf 1)
cs = R.default_corners(W, H)
tx, ty, _ = slow[0]
rows = []
for y in range(ty * 16, min(ty * 16 + 16, H)):
    for x in range(tx * 16, min(tx * 16 + 16, W)):
        xs = np.float32(1.0) - np.float32(x) / np.float32(W - 1)
        ys = np.float32(1.0) - np.float32(y) / np.float32(H - 1)
        o = ys * (xs * cs[0] + (1 - xs) * cs[4]) + (1 - ys) * (xs * cs[2] + (1 - xs) * cs[6])
        dd = ys * (xs * cs[1] + (1 - xs) * cs[5]) + (1 - ys) * (xs * cs[3] + (1 - xs) * cs[7])
        sc.reset_stats()
        sc.set_profiling(True, count_work=True)
        idx, pt = sc.intersect_mesh(o[None].astype(np.float32), dd[None].astype(np.float32))
        w = sc.work_detail(KERNEL_CLOSEST_HIT)
        sh = None
        if idx[0] >= 0:
            so = (pt[0] + np.float32(0.1)).astype(np.float32)
            sc.reset_stats()
            sc.set_profiling(True, count_work=True)
            sc.intersect_mesh(so[None], np.array([wl["lights"][0]], np.float32))
            sh = sc.work_detail(KERNEL_CLOSEST_HIT)
        sc.set_profiling(False)
        # the later bounces of the chain (rt_debug_trace) and their work
        bounces, _ = sc.debug_trace(p, o.astype(np.float32), dd.astype(np.float32))
        later = []
        for b in bounces[1:]:
            sc.reset_stats()
            sc.set_profiling(True, count_work=True)
            sc.intersect_mesh(b["origin"][None], b["dest"][None])
            wb = sc.work_detail(KERNEL_CLOSEST_HIT)
            later.append((b["level"], b["triangle"], wb["visits"], wb["tests"]))
        sc.set_profiling(False)
        rows.append((x, y, int(idx[0]), w["visits"], w["tests"], sh["visits"] if sh else 0, sh["tests"] if sh else 0, later))
rows.sort(key=lambda r: -(r[3] + r[4] + r[5] + r[6] + sum(b[2] + b[3] for b in r[7])))
print(json.dumps({"tile": [tx, ty], "rays": len(rows),
                  "top (x, y, tri, visits, tests, shadow_visits, shadow_tests, [(lvl, tri, visits, tests) of later bounces])": rows[:16],
                  "median_visits": float(np.median([r[3] for r in rows])), "median_tests": float(np.median([r[4] for r in rows]))}))
e = sc.export()
for r in rows[:3]:
    if r[2] >= 0:
        V = e["vertices"][e["triangles"][r[2]]]
        print(json.dumps({"ray_xy": r[:2], "triangle": r[2], "vertices": V.tolist(), "material": int(e["tri_mat"][r[2]])}))
