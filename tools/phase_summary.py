#!/usr/bin/env python3
"""Per-phase VALU breakdown of the four-frame chain launch from rocprofv3 --pmc
runs of tools/phase_probe.py, one directory per variant (gpurun_out/phase/<variant>/<counter set>).
Per variant: the timed instantiation of k_chain (kMulti, not counting), counters summed per dispatch
and averaged over its last `last` dispatches (ordered launches after calibration), per frame (/4).
Phases by subtraction:
  primary walk + shading        = no_shadows_no_secondary
  primary-hit shadow walks      = no_secondary - no_shadows_no_secondary
  secondary walks + shading     = no_shadows - no_shadows_no_secondary
  secondary-hit shadow walks    = all - no_shadows - (primary-hit shadow walks)
  specular (powf, half vector)  = all - no_specular
Usage: python tools/phase_summary.py gpurun_out/phase profiles/r06_valu_phases.json [last]"""
import collections
import csv
import json
import os
import sys

FRAMES = 4


def variant_counters(vdir, last):
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # dispatch -> counter -> value
    names = {}
    for sub in sorted(os.listdir(vdir)):
        for root, _, files in os.walk(os.path.join(vdir, sub)):
            for f in files:
                if not f.endswith("counter_collection.csv"):
                    continue
                for r in csv.DictReader(open(os.path.join(root, f))):
                    n = r["Kernel_Name"]
                    if "k_chain<" not in n:
                        continue
                    targs = n[n.index("<") + 1:n.index(">")].split(",")
                    if len(targs) < 7 or targs[2].strip() != "false" or targs[6].strip() != "true":
                        continue
                    key = (sub, int(r["Dispatch_Id"]))
                    per[key][r["Counter_Name"]] += float(r["Counter_Value"])
                    names[key] = n
    out = {}
    for sub in sorted({k[0] for k in per}):
        ds = sorted(k for k in per if k[0] == sub)[-last:]
        for c in per[ds[0]]:
            out[c] = sum(per[d][c] for d in ds) / len(ds) / FRAMES
        out.setdefault("_dispatches", {})[sub] = len(ds)
    return out


def main(src, dst, last=20):
    v = {d: variant_counters(os.path.join(src, d), last) for d in sorted(os.listdir(src))
         if os.path.isdir(os.path.join(src, d))}
    res = {"what": "per frame (four-frame launches / 4), k_chain<4,true,false,true,false,false,true> (the headline's "
                   "instantiation), counters averaged over each variant's last %d dispatches" % last,
           "variants": v}
    need = ("all", "no_specular", "no_shadows", "no_secondary", "no_shadows_no_secondary")
    if all(n in v for n in need):
        phases = {}
        for c in ("SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_INSTS_SALU",
                  "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS"):
            if not all(c in v[n] for n in need):
                continue
            a, ns, nsh, n2, nn = (v[n][c] for n in need)
            prim_sh = n2 - nn
            phases[c] = {"primary_walk_and_shading": nn, "primary_hit_shadows": prim_sh,
                         "secondary_walks_and_shading": nsh - nn, "secondary_hit_shadows": a - nsh - prim_sh,
                         "specular": a - ns, "total": a}
        for c in phases:
            t = phases[c]["total"]
            phases[c]["share"] = {k: round(x / t, 4) for k, x in phases[c].items() if k != "total"}
        if "SQ_THREAD_CYCLES_VALU" in phases and "SQ_ACTIVE_INST_VALU" in phases:
            phases["lane_utilization"] = {k: round(phases["SQ_THREAD_CYCLES_VALU"][k] / (64 * phases["SQ_ACTIVE_INST_VALU"][k]), 3)
                                          for k in phases["SQ_ACTIVE_INST_VALU"] if k != "share" and phases["SQ_ACTIVE_INST_VALU"][k] > 0}
        res["phases"] = phases
    with open(dst, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res.get("phases", res), indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 20)
