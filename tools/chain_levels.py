#!/usr/bin/env python3
"""Chain-kernel time against chain depth on the benchmark frame: renders C4 with max_lvl 0..3 (and
with shadows off) on one pipeline and prints the chain launch's median time and ray counts, so the
cost of each extra level and of the shadow rays can be read off."""
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
from raytracert_amd._capi import KERNEL_CHAIN, SHADOWS  # noqa: E402

knobs = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
obj = scenes.write_sphere_grid(scenes.C4, tempfile.mkdtemp(), "cl")
sc = R.Scene.load(obj, device=0)
sc.tune("pipes", 1)
for k, v in knobs.items():
    sc.tune(k, v)
for flags in (None, "noshadow"):
    for lvl in range(4):
        p = R.RenderParams(width=1920, height=1080, pf=1, max_lvl=lvl, lights=[[0, 0, 4], [1.5, 1.5, 4]])
        if flags == "noshadow":
            p.flags &= ~SHADOWS
        sc.render(p)
        t = []
        for _ in range(5):
            sc.reset_stats()
            sc.set_profiling(True)
            _, _, counts = sc.render(p)
            sc.set_profiling(False)
            t.append(sc.kernel_stats(KERNEL_CHAIN)[1])
        print(json.dumps({"max_lvl": lvl, "shadows": flags is None, "chain_ms": round(float(np.median(t)), 4),
                          "rays": [int(c) for c in counts]}))
