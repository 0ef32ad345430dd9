#!/usr/bin/env python3
"""Per-step cycle split of bvh4_query (diagnostic build with -DRT_STAMPS via tools/build_ab.sh, loaded
with RTAMD_LIB): node data wait, node arithmetic + stack, triangle data wait, triangle arithmetic,
in shader cycles per lane-visit, for coherent camera rays and incoherent rays leaving the C4
spheres at several batch sizes (the rays of latency_probe.py)."""
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
from raytracert_amd._capi import KERNEL_CLOSEST_HIT, KERNEL_SHADOW  # noqa: E402

obj = scenes.write_sphere_grid(scenes.C4, tempfile.mkdtemp(), "sp")
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


for kind, gen in (("coherent", coherent), ("incoherent", incoherent)):
    for n in (64, 6400, 655360):
        o, d = gen(n)
        sc.intersect_mesh(o, d)
        sc.reset_stats()
        sc.set_profiling(True, count_work=True)
        sc.intersect_mesh(o, d)
        sc.set_profiling(False)
        w = sc.work_detail(KERNEL_CLOSEST_HIT)
        s = sc.work_detail(KERNEL_SHADOW)
        vis, tst = max(w["visits"], 1), max(w["tests"], 1)
        names = list(s.keys())
        st = [s[k] for k in names]
        print(json.dumps({"kind": kind, "n": n, "visits_q": round(vis / n, 2), "tests_q": round(tst / n, 2),
                          "node_wait_cyc": round(st[0] / vis), "node_math_cyc": round(st[1] / vis),
                          "tri_wait_cyc": round(st[2] / tst), "tri_math_cyc": round(st[4] / tst),
                          "query_cyc": round(st[5] / n)}), flush=True)
