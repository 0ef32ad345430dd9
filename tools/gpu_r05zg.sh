#!/bin/bash
# r05: pairing in the closest-hit-shadow kernels (RT_PAIR_CLOSEST 1, built default) vs any-hit only (0): C3 / C4 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
RTAMD_LIB="$PWD/raytracert_amd/ab/lib_b_pairany.so" timeout -k 10 200 python -u tools/pair_diff.py c3 2>&1 | grep -v amdgpu.ids || exit 1
OUT=gpurun_out/r05zg_ab_pair_closest.txt; : > $OUT
for pass in 1 2; do
  for L in raytracert_amd/ab/lib_*.so; do
    for W in c3 c4; do
      echo "== $L $W pass $pass" >> $OUT
      RTAMD_LIB="$PWD/$L" timeout -k 10 200 python -u tools/ab_multi.py $W '[{}]' 2 40 4 >> $OUT 2>&1 || { tail -20 $OUT; exit 1; }
    done
  done
done
grep -v "amdgpu.ids\|^round\|^summary" $OUT | paste - - | cut -c1-200
