#!/bin/bash
# PMC passes with arbitrary counter groups: tools/gpu_pmc_groups.sh TAG "G1;G2;..." [bench args...]
# Each group is one rocprofv3 --kernel-trace --pmc pass (counter limits per block: see
# MI355X_MICROARCH.md) of a short bench run; output under gpurun_out/pmc/TAG/<group>.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; GROUPS_=$2; shift 2
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
IFS=';' read -ra GS <<< "$GROUPS_"
for C in "${GS[@]}"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT/$N" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --no-cpu --profile-steps 1 --no-bf-roofline --pipes 1 "$@" > "$OUT/$N.log" 2>&1 || { echo "pmc $C failed"; tail -5 "$OUT/$N.log"; exit 1; }
done
cd "$GRAFT_REPO_ROOT" && python3 tools/pmc_summary.py "$OUT" "gpurun_out/pmc_$TAG.json" > /dev/null && echo "summary gpurun_out/pmc_$TAG.json"
