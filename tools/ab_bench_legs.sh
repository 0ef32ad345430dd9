#!/bin/bash
# Same-box A/B of bench.py variants on the latency legs (one frame at a time, moving view, cold frame)
# and the headline. Usage: tools/ab_bench_legs.sh TAG PASSES "name[@lib]:extra bench args" ...
# (@lib: raytracert_amd/ab/lib_<lib>.so instead of the in-tree build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; P=$2; shift 2
for pass in $(seq 1 $P); do
  for V in "$@"; do
    N=${V%%:*}; X=${V#*:}
    LIBV=""; case $N in *@*) LIBV=raytracert_amd/ab/lib_${N#*@}.so ;; esac
    R=$(RTAMD_LIB=$LIBV timeout -k 10 300 python bench.py --no-cpu --no-bf-roofline --no-path-compare --no-dropin --no-strong-shares --no-e2e $X 2>gpurun_out/ab_legs_$TAG.err) || { tail -20 gpurun_out/ab_legs_$TAG.err; exit 1; }
    echo "$R" >> gpurun_out/ab_legs_$TAG.jsonl
    echo "$R" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; o=c.get("orbit") or {}; print(sys.argv[1], "pass", sys.argv[2], "head", d["ms_per_step"], "one", (c.get("one_in_flight") or {}).get("ms_per_step"), "orbit1", (o.get("one_in_flight") or {}).get("ms_per_step"), "orbit_vpc", (o.get("views_per_call") or {}).get("ms_per_step"), "cold", c.get("first_frame_ms"), "batch_max", (d.get("batches") or {}).get("max_us"), "mf", {k: v["ms_per_frame"] for k, v in (c.get("multi_frame") or {}).items() if k != "what"})' "$N" "$pass"
  done
done
