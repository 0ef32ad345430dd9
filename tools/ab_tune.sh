#!/bin/bash
# A/B of runtime knobs on the bench's timed loop, alternating, PASSES passes.
# Usage: tools/ab_tune.sh PASSES WORKLOAD "knob=v ..." "knob=v ..." ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
P=$1; WL=$2; shift 2
for pass in $(seq 1 $P); do
  for V in "$@"; do
    A=""; for kv in $V; do A="$A --tune $kv"; done
    R=$(timeout -k 10 200 python bench.py --workload $WL --no-cpu --no-bf-roofline --no-cold --no-path-compare --steps 40 $A 2>/dev/null | tail -1) || exit 1
    echo "$WL [$V] pass $pass $(echo "$R" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms", round(d["value"]), "Mrays/s", "chain", d["kernel_ms_per_step"]["chain"])')"
  done
done
