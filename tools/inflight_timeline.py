#!/usr/bin/env python3
"""k_chain launches from a rocprofv3 kernel-trace CSV in start order: duration, the overlap with the
launch before it (frames in flight: the next frame's launch running beside the previous one's tail)
and the period between launch ends. Prints the last N launches and their means.
    python tools/inflight_timeline.py kernel_trace.csv [N]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_chain" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
seq = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", r.get("Queue_Id", "?"))) for r in rows]
prev_end = None
out = []
for st, en, q in seq[-n:]:
    ov = max(0, prev_end - st) if prev_end is not None else 0
    per = en - prev_end if prev_end is not None else 0
    out.append((st, en, q, ov, per))
    prev_end = en if prev_end is None else max(prev_end, en)
t0 = out[0][0]
for st, en, q, ov, per in out:
    print(f"start {(st - t0) / 1e3:9.1f} us  dur {(en - st) / 1e3:7.1f} us  overlap {ov / 1e3:6.1f} us  end-to-end {per / 1e3:6.1f} us  queue {q}")
k = len(out) - 1
if k > 0:
    print(f"mean dur {sum(e - s for s, e, *_ in out) / len(out) / 1e3:.1f} us, mean overlap {sum(o[3] for o in out[1:]) / k / 1e3:.1f} us, "
          f"mean period {(out[-1][1] - out[0][1]) / k / 1e3:.1f} us")
