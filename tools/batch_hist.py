"""Distribution of the wave-batch lifetimes of an ordered frame (r05 critical-path diagnostic).

Renders warm frames of a bench workload one at a time, then prints for the last few launches how
many batches live longer than each threshold, the share of the frame's summed batch time they
hold, and saves the durations (and the batch order's head) as .npy under gpurun_out/.
Usage: python tools/batch_hist.py [workload] [frames]
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402


def main():
    wl_name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    wl = bench.WORKLOADS[wl_name]
    out_dir = os.path.join(os.path.dirname(HERE), "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    with tempfile.TemporaryDirectory() as d:
        path = bench.workload_scene(wl["scene"], d)
        p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"],
                           lights=[list(x) for x in wl["lights"]])
        with R.Scene.load(path, device=0) as sc:
            for kv in filter(None, os.environ.get("RT_CRIT_TUNE", "").split(",")):
                k, v = kv.split("=")
                sc.tune(k, int(v))
            for _ in range(frames):
                sc.render(p)
            print("trials:", sc.trials())
            runs = []
            for i in range(3):
                sc.render(p)
                runs.append(sc.batch_durations().astype(np.float64))
            np.save(os.path.join(out_dir, f"batch_durations_{wl_name}.npy"), np.stack(runs))
            for dur in runs:
                s = np.sort(dur)[::-1]
                tot = s.sum()
                line = [f"n {s.size} max {s[0]:.1f} sum {tot / 1e3:.2f} ms"]
                for thr in (350, 300, 250, 200, 150, 100, 50):
                    k = int((s > thr).sum())
                    line.append(f">{thr}us: {k} ({s[:k].sum() / tot * 100:.1f}%)")
                print("  ".join(line))
                print("   top ranks:", " ".join(f"{r}:{s[r]:.0f}" for r in (0, 8, 32, 64, 128, 256, 512, 1024, 2048, 4096)
                                                 if r < s.size))


if __name__ == "__main__":
    main()
