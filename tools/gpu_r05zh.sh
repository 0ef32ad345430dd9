#!/bin/bash
# r05: table-driven spec_pow (RT_SPEC_POW_TABLE 1) vs the atanh / degree-14 form: A/B, then the GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/r05zh_ab_spec_table.txt; : > $OUT
for pass in 1 2; do
  for L in raytracert_amd/ab/lib_*.so; do
    for W in c4 c5 ref_default; do
      echo "== $L $W pass $pass" >> $OUT
      RTAMD_LIB="$PWD/$L" timeout -k 10 200 python -u tools/ab_multi.py $W '[{}]' 2 $([ $W = c5 ] && echo 6 || echo 40) 4 >> $OUT 2>&1 || { tail -20 $OUT; exit 1; }
    done
    echo "== $L c4-single pass $pass" >> $OUT
    RTAMD_LIB="$PWD/$L" timeout -k 10 200 python -u tools/ab_frame.py c4 '[{"chain_split": 5, "wave_steal": 2, "steal_quarter": -1, "shadow_helpers": 2}]' 2 40 >> $OUT 2>&1 || { tail -20 $OUT; exit 1; }
  done
done
grep -v "amdgpu.ids\|^round\|^summary" $OUT | paste - - | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r05zh_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05zh_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05zh_pytest_gpu.log
