#!/bin/bash
# One PMC pass (counter set $1) per A/B library raytracert_amd/ab/lib_*.so, on the bench's chain
# kernel: gpurun_out/${PMC_OUT:-pmc_ab}/<lib>/... (summarise with tools/pmc_ab_summary.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
C=${1:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD"}
OUT="$GRAFT_REPO_ROOT/gpurun_out/${PMC_OUT:-pmc_ab}"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import torch" || exit 1
for L in raytracert_amd/ab/lib_*.so; do
  N=$(basename $L .so)
  RTAMD_LIB="$GRAFT_REPO_ROOT/$L" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT/$N" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 2 --no-cpu --no-cold --no-path-compare --profile-steps 1 --no-bf-roofline --pipes 1 > "$OUT/$N.log" 2>&1 || { echo "pmc $N failed"; tail -5 "$OUT/$N.log"; exit 1; }
done
