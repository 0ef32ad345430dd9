#!/usr/bin/env python3
"""Wave-level iteration counts of the chain kernel's regions and the lanes active in them, from a
-DRT_REGION_COUNTS build (tools/build_ab.sh rc "-DRT_REGION_COUNTS"), on one ordered frame of a
workload with the plain (non-stealing) walk:

    WORKLOAD=c4 RTAMD_LIB=raytracert_amd/ab/lib_rc.so python tools/region_counts.py
"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import torch  # noqa: E402,F401

import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402

wl = bench.WORKLOADS[os.environ.get("WORKLOAD", "c4")]
obj = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
sc = R.Scene.load(obj, device=0)
sc.tune("wave_steal", 0)
p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl.get("pf", 1), max_lvl=wl["max_lvl"], lights=wl["lights"])
for _ in range(3):
    sc.render(p)
sc.reset_stats()
sc.set_profiling(True, count_work=True)
sc.render(p)
sc.set_profiling(False)
d = [int(v) for v in sc.diag_read(0, 32)]
names = ["chain_step", "closest_query", "shadow_query", "closest_node_iter", "closest_leaf_iter",
         "shadow_node_iter", "shadow_leaf_iter", "shade"]
out = {n: {"wave_iters": d[i], "active_lanes": d[16 + i], "lane_util": round(d[16 + i] / max(64 * d[i], 1), 3)}
       for i, n in enumerate(names)}
print(json.dumps({"workload": os.environ.get("WORKLOAD", "c4"), "regions": out}, indent=1))
