#!/usr/bin/env python3
"""Per-kernel launch statistics from a rocprofv3 --kernel-trace run (the *_kernel_trace.csv under
the -d directory): launches, mean, median, and the mean over launches after the first `skip` of
each kernel (the first launches of a view run before a batch order exists).

    python tools/kernel_trace_summary.py gpurun_out/prof/r02 [skip] > profiles/r02_kernel_trace_summary.json
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def main(root, skip=3):
    files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {root}")
    durs = collections.defaultdict(list)
    for f in files:
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            name = r["Kernel_Name"].replace("rt::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            durs[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)   # us
    out = {}
    for k, d in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        tail = d[skip:] if len(d) > skip else d
        out[k] = {"launches": len(d), "mean_us": round(statistics.fmean(d), 2), "median_us": round(statistics.median(d), 2),
                  "min_us": round(min(d), 2), "max_us": round(max(d), 2),
                  f"mean_after_first_{skip}_us": round(statistics.fmean(tail), 2), "total_us": round(sum(d), 1)}
    json.dump({"source": root, "skip": skip, "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
