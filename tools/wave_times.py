#!/usr/bin/env python3
"""Wave residency of the chain launch over time (diagnostic build with -DRT_WAVE_TIMES, loaded via
RTAMD_LIB): renders the C4 frame on one pipeline in counting mode, reads each wave's start/end
clock (100 MHz) and query count, and prints how many waves are alive across the launch."""
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

knobs = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
import bench  # noqa: E402  (WORKLOAD=c2|c3|c4|c5: the bench's configurations)
wl = bench.WORKLOADS[os.environ.get("WORKLOAD", "c4")]
obj = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
sc = R.Scene.load(obj, device=0)
sc.tune("pipes", 1)
for k, v in knobs.items():
    sc.tune(k, v)
p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=int(os.environ.get("MAX_LVL", wl["max_lvl"])),
                   lights=wl["lights"])
sc.render(p)
sc.reset_stats()
sc.set_profiling(True, count_work=True)
sc.render(p)
sc.set_profiling(False)
d = sc.diag_read(0, 3 * 43690).reshape(-1, 3).astype(np.int64)
d = d[d[:, 1] > 0]
t0 = d[:, 0].min()
s, e = (d[:, 0] - t0) * 0.01, (d[:, 1] - t0) * 0.01   # microseconds
span = e.max()
bins = np.linspace(0, span, 21)
alive = [int(((s <= b) & (e > b)).sum()) for b in bins[:-1]]
life = e - s
print(json.dumps({"waves": len(d), "span_us": round(float(span), 1), "alive_at_5pct_steps": alive,
                  "life_us_pcts": [round(float(np.percentile(life, q)), 1) for q in (5, 25, 50, 75, 95, 100)],
                  "start_us_pcts": [round(float(np.percentile(s, q)), 1) for q in (5, 25, 50, 75, 95, 100)],
                  "end_us_pcts": [round(float(np.percentile(e, q)), 1) for q in (5, 25, 50, 75, 95, 100)],
                  "queries_per_wave_pcts": [int(np.percentile(d[:, 2] & 0xFFFFFFFF, q)) for q in (5, 50, 95, 100)]}))
# who finishes first: lifetime by dispatch order (start-time deciles) and, per SIMD, the order in
# which its waves end (rank of each wave's end among the waves that shared its SIMD)
order = np.argsort(s, kind="stable")
dec = np.array_split(order, 10)
print(json.dumps({"life_us_by_start_decile": [round(float(life[i].mean()), 1) for i in dec]}))
hw = (d[:, 2] >> 32) & 0x0FFFFFFF
xcc = (d[:, 2] >> 60) & 0xF
simd = (xcc << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 8) & 0xF) << 4) | ((hw >> 4) & 3)
groups = {}
for i, g in enumerate(simd):
    groups.setdefault(int(g), []).append(i)
sizes = [len(v) for v in groups.values()]
ends_by_rank = {}
for v in groups.values():
    v = sorted(v, key=lambda i: s[i])   # by start on this SIMD
    for r, i in enumerate(v):
        ends_by_rank.setdefault(r, []).append(e[i])
print(json.dumps({"simds": len(groups), "waves_per_simd_pcts": [int(np.percentile(sizes, q)) for q in (5, 50, 95)],
                  "mean_end_us_by_start_rank_on_simd": {r: round(float(np.mean(x)), 1) for r, x in sorted(ends_by_rank.items()) if len(x) > 50}}))
# where the long waves are: wave w takes samples [64 w, 64 w + 64) of the tile-major queue
# (one batch per wave when the grid covers the frame); map them to 16x16 tiles on the screen
if len(d) * 64 >= p.width * p.height:
    tiles_x = (p.width + 15) // 16
    order = np.argsort(-life)
    top = [(int(i) * 64 // 256 % tiles_x, int(i) * 64 // 256 // tiles_x, round(float(life[i]), 1)) for i in order[:20]]
    print(json.dumps({"slowest_waves_tile_xy_us": top}))
    tiles_y = (p.height + 15) // 16
    grid = np.zeros((tiles_y, tiles_x))
    for i in range(len(d)):
        t = i * 64 // 256
        if t < tiles_x * tiles_y:
            grid[t // tiles_x, t % tiles_x] = max(grid[t // tiles_x, t % tiles_x], life[i])
    coarse = grid[: tiles_y // 6 * 6, : tiles_x // 10 * 10].reshape(tiles_y // 6, 6, tiles_x // 10, 10).max(axis=(1, 3))
    print("max wave life (us) per 160x96-pixel block:")
    for row in coarse:
        print(" ".join(f"{v:5.0f}" for v in row))
