#!/bin/bash
# PMC passes for the closest-hit kernel's HBM traffic (MI355X_MICROARCH.md §HBM: FETCH_SIZE and
# WRITE_SIZE in separate passes, kernel trace only; FETCH_SIZE reads 1/2 of wide streaming reads).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 python3 -c "import torch" || exit 1
# WORKLOAD (optional): bench workload to profile (default c4).
WL_ARG=""; [ -n "$WORKLOAD" ] && WL_ARG="--workload $WORKLOAD"
# PMC_SETS (optional): counter sets separated by ';' instead of the default traffic passes.
if [ -n "$PMC_SETS" ]; then IFS=';' read -ra SETS <<< "$PMC_SETS"; else
SETS=(FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU"); fi
for C in "${SETS[@]}"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT/$N" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 8 --warmup 30 --inflight 1 --no-cpu --no-cold --no-path-compare --profile-steps 1 --no-bf-roofline --no-dropin --pipes 1 --orbit-step 0 --no-multi-frame --no-strong-shares --no-e2e $WL_ARG > "$OUT/$N.log" 2>&1 || { echo "pmc $C failed"; tail -5 "$OUT/$N.log"; exit 1; }
done
ls -R "$OUT" > "$OUT/listing.txt"
