"""Critical-path diagnostic: the longest wave batches of an ordered frame, re-rendered alone.

For a workload of bench.py, renders warm frames, takes the per-batch wave lifetimes
(rt_batch_durations), and re-renders each of the longest batches' pixel rectangles by themselves
(an otherwise idle GPU): if a batch is as slow alone as inside the frame, its time is the latency
of its own chains (walk iterations x load latency); if much faster, it is contention with the rest
of the frame. Also prints the work counters (rays, node visits, triangle tests) of each rectangle.
Usage: python tools/critical_path.py [workload] [n_longest]
RT_CRIT_TUNE='knob=v,knob=v' applies Scene.tune knobs first (e.g. wave_steal=1,split_eighth=512).
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402
from raytracert_amd import _capi  # noqa: E402


def main():
    wl_name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    n_top = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    wl = bench.WORKLOADS[wl_name]
    tile = 16
    spp = wl["pf"] * wl["pf"]
    spb = (64 // spp) * spp
    with tempfile.TemporaryDirectory() as d:
        path = bench.workload_scene(wl["scene"], d)
        p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"],
                           lights=[list(x) for x in wl["lights"]])
        with R.Scene.load(path, device=0) as sc:
            for kv in filter(None, os.environ.get("RT_CRIT_TUNE", "").split(",")):
                k, v = kv.split("=")
                sc.tune(k, int(v))
            for _ in range(8):
                sc.render(p)
            dur = sc.batch_durations()
            print(f"{wl_name}: {dur.size} batches, max {dur.max():.1f} us, p99 {np.percentile(dur, 99):.1f}, "
                  f"median {np.median(dur):.1f}, sum {dur.sum() / 1e3:.1f} ms")
            tiles_x = (wl["width"] + tile - 1) // tile
            # pixel order in a tile (RT_TUNE_PIXEL_ORDER auto): Morton unless the launch may steal
            morton = wl["width"] * wl["height"] * spp > 2 * R.device_resident_lanes() if hasattr(R, "device_resident_lanes") \
                else int(os.environ.get("RT_CRIT_MORTON", "1"))

            def pixel_xy(pix):
                t, q = divmod(pix, tile * tile)
                ty, tx = divmod(t, tiles_x)
                if morton:
                    px = sum(((q >> (2 * k)) & 1) << k for k in range(8))
                    py = sum(((q >> (2 * k + 1)) & 1) << k for k in range(8))
                else:
                    py, px = divmod(q, tile)
                return tx * tile + px, ty * tile + py

            for b in np.argsort(dur)[::-1][:n_top]:
                s0 = int(b) * spb   # first sample of the batch (tile-major, 16 x 16 tiles, spp per pixel)
                xy = [pixel_xy(q) for q in range(s0 // spp, (s0 + spb - 1) // spp + 1)]
                x0, y0 = min(v[0] for v in xy), min(v[1] for v in xy)
                rect = (x0, y0, max(v[0] for v in xy) - x0 + 1, max(v[1] for v in xy) - y0 + 1)
                alone = []
                for _ in range(4):
                    sc.render(p, *rect)
                    alone.append(float(sc.batch_durations().max()))
                sc.reset_stats()
                sc.set_profiling(True, count_work=True)
                _, _, counts = sc.render(p, *rect)
                sc.set_profiling(False)
                ct, cv = sc.work_stats(_capi.KERNEL_CLOSEST_HIT)
                st, sv = sc.work_stats(_capi.KERNEL_SHADOW)
                print(f"  batch {int(b)}: {dur[b]:.1f} us in the frame; alone {min(alone):.1f}-{max(alone):.1f} us; "
                      f"rect {rect}; rays {[int(c) for c in counts]}; closest visits {cv:.0f} tests {ct:.0f}; shadow visits {sv:.0f} tests {st:.0f}")


if __name__ == "__main__":
    main()
