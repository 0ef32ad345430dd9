#!/usr/bin/env python3
"""Print one frame's kernel timeline from a rocprofv3 kernel-trace CSV (second frame rendered)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seq = [(r['Kernel_Name'].replace('rt::(anonymous namespace)::', '').split('(')[0].replace('void ', ''),
        (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, int(r['Grid_Size_X']),
        int(r['Start_Timestamp']), r['VGPR_Count'], r['LDS_Block_Size']) for r in rows]
seq = [x for x in seq if x[0].startswith('k_')]
starts = [i for i, x in enumerate(seq) if x[0] == 'k_gen_primary']
which = int(sys.argv[2]) if len(sys.argv) > 2 else 1
i0, i1 = starts[which], (starts[which + 1] if which + 1 < len(starts) else len(seq))
t0 = seq[i0][3]
tot = {}
for name, us, grid, st, vg, lds in seq[i0:i1]:
    print(f"{name:28s} {us:8.1f} us grid {grid:9d} vgpr {vg:>4} lds {lds:>6} t={(st - t0) / 1e3:8.1f}")
    tot[name] = tot.get(name, 0) + us
print('frame span us', (seq[i1 - 1][3] - t0) / 1e3 + seq[i1 - 1][1])
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {v:8.1f} us")
