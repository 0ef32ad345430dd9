#!/usr/bin/env python3
"""Per-launch PMC counters of the production chain kernel (k_chain<4,true,false,true>) for each
A/B library of tools/pmc_ab.sh, excluding its first (unordered) launch; kernel time from the
same trace. Usage: python tools/pmc_ab_summary.py [gpurun_out/pmc_ab]"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_ab"
res = {}
for d in sorted(glob.glob(os.path.join(root, "lib_*"))):
    if not os.path.isdir(d):
        continue
    rows = [r for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            for r in csv.DictReader(open(f))]
    # the production chain kernel: k_chain<4, true, false, true[, steal]> with the plain walk
    prod = [r for r in rows if "k_chain<4, true, false, true" in r["Kernel_Name"] and "true, false, true, true" not in r["Kernel_Name"]]
    disp = sorted({int(r["Dispatch_Id"]) for r in prod})[1:]   # drop the first launch
    acc = collections.defaultdict(float)
    for r in prod:
        if int(r["Dispatch_Id"]) in disp:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
    n = max(len(disp), 1)
    tr = [r for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True) for r in csv.DictReader(open(f))
          if "k_chain<4, true, false, true" in r["Kernel_Name"] and int(r["Dispatch_Id"]) in disp]
    us = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tr) / max(len(tr), 1)
    res[os.path.basename(d)] = {"launches": len(disp), "kernel_us": round(us, 1), **{k: round(v / n) for k, v in sorted(acc.items())}}
print(json.dumps(res, indent=1))
