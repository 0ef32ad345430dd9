#!/usr/bin/env python3
"""Per-frame timeline from a rocprofv3 kernel-trace CSV of bench.py, every dispatch included
(runtime fills/copies too): the gaps between launches are the frame's fixed cost.
    python tools/frame_gaps.py run_kernel_trace.csv [frame_index]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].replace("rt::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40],
        int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
starts = [i for i, x in enumerate(seq) if x[0] == "k_gen_primary"]
which = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
i0, i1 = starts[which], starts[which + 1] if which + 1 < len(starts) else len(seq)
t0 = seq[i0][1]
prev_end = t0
for name, st, en in seq[i0:i1]:
    print(f"{name:40s} start {(st - t0) / 1e3:8.1f} us  dur {(en - st) / 1e3:8.1f} us  gap {(st - prev_end) / 1e3:6.1f} us")
    prev_end = max(prev_end, en)
print(f"frame period {(seq[i1][1] - t0) / 1e3 if i1 < len(seq) else float('nan'):.1f} us")
