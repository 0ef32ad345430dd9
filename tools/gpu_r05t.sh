#!/bin/bash
# r05: the negligible-specular skip (RT_SPEC_SKIP), multi-frame launches,
# hit), then the full GPU suite on the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/r05t_ab_spec_skip.txt; : > $OUT
for pass in 1 2; do
  for L in raytracert_amd/ab/lib_*.so; do
    for W in c4 c5; do
      echo "== $L $W pass $pass" >> $OUT
      RTAMD_LIB="$PWD/$L" timeout -k 10 200 python -u tools/ab_multi.py $W '[{}]' 2 $([ $W = c5 ] && echo 6 || echo 40) 4 >> $OUT 2>&1 || { tail -20 $OUT; exit 1; }
    done
  done
done
grep -A1 "^==\|summary" $OUT | grep "==\|ms per frame" | grep -v round
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r05t_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05o_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05t_pytest_gpu.log
