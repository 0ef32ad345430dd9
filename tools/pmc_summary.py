#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh) into profiles/<tag>_pmc.json.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from
separate passes (they do not fit one pass), both in KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide streaming reads, so it is doubled before adding WRITE_SIZE. bench.py reports the
`traffic_bytes_per_launch` of the kernel it rooflines from the newest summary for the same kernel.

    python tools/pmc_summary.py gpurun_out/pmc/r01 profiles/r01_pmc.json
"""
import collections
import csv
import json
import os
import sys


def load(pass_dir):
    rows = list(csv.DictReader(open(os.path.join(pass_dir, "run_counter_collection.csv"))))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        name = r["Kernel_Name"]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
    return agg, disp


def main(src, dst):
    kernels = collections.defaultdict(dict)
    for d in sorted(os.listdir(src)):
        p = os.path.join(src, d)
        if not os.path.isdir(p) or not os.path.exists(os.path.join(p, "run_counter_collection.csv")):
            continue
        agg, disp = load(p)
        for name, counters in agg.items():
            if not name.startswith("rt::") and "rt::" not in name:
                continue
            short = name.replace("rt::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            n = len(disp[name])
            for c, v in counters.items():
                kernels[short][c + "_per_launch"] = v / n
            kernels[short]["launches_in_pass"] = n
    for k, c in kernels.items():
        if "FETCH_SIZE_per_launch" in c and "WRITE_SIZE_per_launch" in c:
            c["traffic_bytes_per_launch"] = (2.0 * c["FETCH_SIZE_per_launch"] + c["WRITE_SIZE_per_launch"]) * 1024.0
        if "TCC_HIT_sum_per_launch" in c and "TCC_MISS_sum_per_launch" in c:
            h, m = c["TCC_HIT_sum_per_launch"], c["TCC_MISS_sum_per_launch"]
            c["l2_hit_rate"] = h / max(h + m, 1.0)
    out = {"source": os.path.abspath(src), "method": "rocprofv3 --kernel-trace --pmc, one pass per counter group; "
           "traffic = (2*FETCH_SIZE + WRITE_SIZE) KiB per launch (gfx950 FETCH_SIZE halving corrected)",
           "kernels": kernels}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
