#!/usr/bin/env python3
"""Per-chain-step cost of the benchmark frame: renders with max_lvl = 0..L and differences the
per-kind kernel times, queue sizes and BVH work counters, so each step's closest-hit and shadow
launches can be read against their query counts (median of `rounds` timed renders per level)."""
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

knobs = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
spec = getattr(scenes, sys.argv[3]) if len(sys.argv) > 3 else scenes.C4
obj = scenes.write_sphere_grid(spec, tempfile.mkdtemp(), "sp")
sc = R.Scene.load(obj, device=0)
for k, v in knobs.items():
    sc.tune(k, v)
rows = []
for lvl in range(0, 4):
    p = R.RenderParams(width=1920, height=1080, pf=1, max_lvl=lvl, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    sc.render(p)
    t = []
    for _ in range(rounds):
        sc.reset_stats()
        sc.set_profiling(True)
        _, _, counts = sc.render(p)
        sc.set_profiling(False)
        t.append((sc.kernel_stats(KERNEL_CLOSEST_HIT)[1], sc.kernel_stats(KERNEL_SHADOW)[1]))
    sc.reset_stats()
    sc.set_profiling(True, count_work=True)
    sc.render(p)
    sc.set_profiling(False)
    ch_q = sc.kernel_stats(KERNEL_CLOSEST_HIT)[2] / sc.counts()[1]
    sh_q = sc.kernel_stats(KERNEL_SHADOW)[2] / sc.counts()[1]
    rows.append(dict(lvl=lvl, ch_ms=float(np.median([x[0] for x in t])), sh_ms=float(np.median([x[1] for x in t])),
                     ch_q=ch_q, sh_q=sh_q, ch=sc.work_detail(KERNEL_CLOSEST_HIT), sh=sc.work_detail(KERNEL_SHADOW)))
prev = None
for r in rows:
    d = dict(step=r["lvl"])
    for kind in ("ch", "sh"):
        pr = prev or {f"{kind}_ms": 0.0, f"{kind}_q": 0.0, kind: {k: 0 for k in r[kind]}}
        ms = r[f"{kind}_ms"] - pr[f"{kind}_ms"]
        q = r[f"{kind}_q"] - pr[f"{kind}_q"]
        w = {k: r[kind][k] - pr[kind][k] for k in ("tests", "visits", "wave_max_visits", "wave_tasks", "wave_max_tests")}
        d[kind] = dict(ms=round(ms, 4), queries=int(q), ns_per_query=round(ms * 1e6 / max(q, 1), 3),
                       visits_per_q=round(w["visits"] / max(q, 1), 2), tests_per_q=round(w["tests"] / max(q, 1), 2),
                       wave_tasks=w["wave_tasks"],
                       steps_per_task=round((w["wave_max_visits"] + w["wave_max_tests"]) / max(w["wave_tasks"], 1), 2),
                       simd_eff=round(w["visits"] / max(64 * w["wave_max_visits"], 1), 3),
                       max_visits=r[kind]["max_visits"])
    print(json.dumps(d))
    prev = r
