#!/bin/bash
# A/B of the split of the longest batches of ordered chain launches (RT_TUNE_STEAL_HALF /
# _QUARTER / RT_TUNE_SPLIT_EIGHTH) and their wave priority (RT_TUNE_PRIORITY_BATCHES) on the
# bench's timed loop, variants alternating.
# Usage: tools/ab_split.sh PASSES WORKLOAD "half quarter eighth prio [extra bench args]" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
P=$1; W=$2; shift 2
VARIANTS=("$@")
for pass in $(seq 1 $P); do
  for V in "${VARIANTS[@]}"; do
    read -r H Q E PR X <<< "$V"
    R=$(timeout -k 10 200 python bench.py --workload $W --no-cpu --no-bf-roofline --no-cold --no-path-compare --no-dropin \
        --steps 100 --tune steal_half=$H --tune steal_quarter=$Q --tune split_eighth=$E --tune prio_batches=$PR $X \
        2>gpurun_out/ab_last.err) || exit 1
    echo "$W half=$H quarter=$Q eighth=$E prio=$PR $X pass $pass $(echo "$R" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d.get("batches") or {}; print(d["ms_per_step"], "ms", "batch max", b.get("max_us"), "p99", b.get("p99_us"), "sum", b.get("sum_ms"))')"
  done
done
