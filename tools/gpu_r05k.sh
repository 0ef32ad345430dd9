#!/bin/bash
# r05: node-visit variants (r04's within-noise cuts) re-measured where the VALU binds: 4 frames per
# call (multi-frame launch, VALU busy ~0.99). Builds from tools/build_ab.sh, alternating passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/r05k_ab_node_multi.txt; : > $OUT
for pass in 1 2; do
  for L in raytracert_amd/ab/lib_*.so; do
    echo "== $L pass $pass" >> $OUT
    RTAMD_LIB="$PWD/$L" timeout -k 10 200 python -u tools/ab_multi.py c4 '[{}]' 3 60 4 >> $OUT 2>&1 || { tail -20 $OUT; exit 1; }
  done
done
grep -A1 "^==\|summary" $OUT | grep "==\|ms per frame" | grep -v round
