#!/usr/bin/env python3
"""Latency of the BVH traversal at low occupancy: intersect_mesh on batches of 64 ... 655,360
incoherent rays that start on the C4 spheres (like the chain's late reflection steps) and on
coherent camera rays. Run under `rocprofv3 --kernel-trace` to get each launch's duration; the
work counters give visits and tests per query (their wave maxima bound the serial steps)."""
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
from raytracert_amd._capi import KERNEL_CLOSEST_HIT  # noqa: E402

obj = scenes.write_sphere_grid(scenes.C4, tempfile.mkdtemp(), "lp")
sc = R.Scene.load(obj, device=0)
e = sc.export()
V, F = e["vertices"], e["triangles"]
rng = np.random.default_rng(1)
cs = R.default_corners(1920, 1080)


def incoherent(n):
    t = rng.integers(0, len(F) - 2, n)
    P = V[F[t]].mean(1)
    nrm = e["normals"][t]
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1)[:, None]
    d = np.where((d * nrm).sum(1)[:, None] < 0, -d, d)
    o = (P + 0.01 * nrm).astype(np.float32)
    return o, (o + d).astype(np.float32)


def coherent(n):
    side = int(np.ceil(np.sqrt(n)))
    a, b = np.meshgrid(np.linspace(0.3, 0.7, side), np.linspace(0.3, 0.7, side))
    a, b = a.reshape(-1)[:n, None].astype(np.float32), b.reshape(-1)[:n, None].astype(np.float32)
    o = (cs[0] * a + cs[4] * (1 - a)) * b + (cs[2] * a + cs[6] * (1 - a)) * (1 - b)
    d = (cs[1] * a + cs[5] * (1 - a)) * b + (cs[3] * a + cs[7] * (1 - a)) * (1 - b)
    return o.astype(np.float32), d.astype(np.float32)


knobs = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
for k, v in knobs.items():
    sc.tune(k, v)
for kind, gen in (("incoherent", incoherent), ("coherent", coherent)):
    for n in (64, 640, 6400, 64000, 655360):
        o, d = gen(n)
        sc.intersect_mesh(o, d)          # timed launches: read the kernel trace, 3 per size
        sc.intersect_mesh(o, d)
        sc.intersect_mesh(o, d)
        sc.reset_stats()
        sc.set_profiling(True, count_work=True)
        sc.intersect_mesh(o, d)
        sc.set_profiling(False)
        w = sc.work_detail(KERNEL_CLOSEST_HIT)
        print(json.dumps({"kind": kind, "n": n, "visits_q": round(w["visits"] / n, 2), "tests_q": round(w["tests"] / n, 2),
                          "max_visits": w["max_visits"],
                          "steps_per_task": round((w["wave_max_visits"] + w["wave_max_tests"]) / max(w["wave_tasks"], 1), 1)}),
              flush=True)
