#!/bin/bash
# r05: the triangle test's s, t divisions from the record's reciprocal slot (RT_TRI_RCP 1):
# exhaustive significand check of the Markstein correction, the GPU suite, then an A/B against RT_TRI_RCP 0.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 tools/bin/markstein_gpu control > gpurun_out/r05zi_markstein_gpu.txt 2>&1 || { tail -5 gpurun_out/r05zi_markstein_gpu.txt; exit 1; }
tail -3 gpurun_out/r05zi_markstein_gpu.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r05zi_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05zi_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05zi_pytest_gpu.log
OUT=gpurun_out/r05zi_ab_tri_rcp.txt; : > $OUT
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
