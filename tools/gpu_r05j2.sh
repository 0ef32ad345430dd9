#!/bin/bash
# r05: waves per EU of the multi-frame chain kernel (RT_MULTI_WPE 4 / 5 / 6), four frames per call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/r05j2_ab_multi_wpe.txt; : > $OUT
for pass in 1 2; do
  for L in raytracert_amd/ab/lib_*.so; do
    for W in c4 c5 ref_default; do
      echo "== $L $W pass $pass" >> $OUT
      RTAMD_LIB="$PWD/$L" timeout -k 10 200 python -u tools/ab_multi.py $W '[{}]' 2 $([ $W = c5 ] && echo 6 || echo 40) 4 >> $OUT 2>&1 || { tail -20 $OUT; exit 1; }
    done
  done
done
grep -v "amdgpu.ids\|^round\|^summary" $OUT | paste - -
