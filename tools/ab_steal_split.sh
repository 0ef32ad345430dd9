#!/bin/bash
# A/B of the stealing kernel's split of the longest batches (RT_TUNE_STEAL_HALF / _QUARTER) on
# the bench's timed loop, C2 and C3, variants alternating. Usage: tools/ab_steal_split.sh [PASSES]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
P=${1:-2}
for pass in $(seq 1 $P); do
  for W in c2 c3; do
    for V in "512 0" "512 4" "512 16" "512 64" "0 64" "0 256"; do
      set -- $V
      R=$(timeout -k 10 200 python bench.py --workload $W --no-cpu --no-bf-roofline --no-cold --no-path-compare \
          --steps 200 --tune steal_half=$1 --tune steal_quarter=$2 2>/dev/null) || exit 1
      echo "$W half=$1 quarter=$2 pass $pass $(echo "$R" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms", "chain", d["kernel_ms_per_step"]["chain"])')"
    done
  done
done
