#!/bin/bash
# A/B of kernel builds: tools/ab_tune.py against each raytracert_amd/ab/lib_*.so in turn (RTAMD_LIB),
# two passes in alternating order. Usage: tools/ab_libs.sh '<variants json>' ROUNDS [SCENE]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=${1:-'[{}]'}; R=${2:-5}; S=${3:-C4}
for pass in 1 2; do
  for L in raytracert_amd/ab/lib_*.so; do
    echo "== $L pass $pass"
    RTAMD_LIB="$PWD/$L" timeout -k 10 200 python tools/ab_tune.py "$V" "$R" "$S" 2>/dev/null | cut -c1-200 || exit 1
  done
done
