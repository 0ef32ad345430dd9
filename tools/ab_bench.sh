#!/bin/bash
# A/B of whole builds on the bench's own timed loop (many frames back to back): bench.py against
# each raytracert_amd/ab/lib_*.so in turn (RTAMD_LIB), alternating, PASSES passes.
# Usage: tools/ab_bench.sh [PASSES] [extra bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
P=${1:-2}; shift
for pass in $(seq 1 $P); do
  for L in raytracert_amd/ab/lib_*.so; do
    R=$(RTAMD_LIB="$PWD/$L" timeout -k 10 200 python bench.py --no-cpu --no-bf-roofline --no-cold --no-path-compare --steps 40 "$@" 2>gpurun_out/ab_last.err) || { tail -5 gpurun_out/ab_last.err; exit 1; }
    echo "$L pass $pass $(echo "$R" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms", round(d["value"]), "Mrays/s", "chain", d["kernel_ms_per_step"]["chain"])')"
  done
done
