#!/bin/bash
# r05: record stores without sc1 (RT_CHAIN_SC1 0) and plain pops (RT_POP_FAST 0) under the multi-frame launch: A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/r05zm_ab_sc1_pop.txt; : > $OUT
for pass in 1 2; do
  for L in raytracert_amd/ab/lib_*.so; do
    for W in c4 c5 ref_default c3; do
      echo "== $L $W pass $pass" >> $OUT
      RTAMD_LIB="$PWD/$L" timeout -k 10 200 python -u tools/ab_multi.py $W '[{}]' 2 $([ $W = c5 ] && echo 6 || echo 40) 4 >> $OUT 2>&1 || { tail -20 $OUT; exit 1; }
    done
    echo "== $L c4-single pass $pass" >> $OUT
    RTAMD_LIB="$PWD/$L" timeout -k 10 200 python -u tools/ab_frame.py c4 '[{"chain_split": 5, "wave_steal": 2, "steal_quarter": -1, "shadow_helpers": 2}]' 2 40 >> $OUT 2>&1 || { tail -20 $OUT; exit 1; }
  done
done
grep -v "amdgpu.ids\|^round\|^summary" $OUT | paste - - | cut -c1-200
