#!/bin/bash
# r05: up to 8 frames per call: parity, then C4 and the reference's defaults at 4 and 8 frames per call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiframe.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05n_pytest.log 2>&1 || { tail -30 gpurun_out/r05n_pytest.log; exit 1; }
tail -2 gpurun_out/r05n_pytest.log
for W in c4 ref_default; do
  timeout -k 10 300 python -u tools/ab_multi.py $W '[{}]' 3 40 4 > gpurun_out/r05n_ab_k4_$W.txt 2>&1 || { tail -20 gpurun_out/r05n_ab_k4_$W.txt; exit 1; }
  timeout -k 10 300 python -u tools/ab_multi.py $W '[{}]' 3 20 8 > gpurun_out/r05n_ab_k8_$W.txt 2>&1 || { tail -20 gpurun_out/r05n_ab_k8_$W.txt; exit 1; }
  echo "$W K=4: $(tail -1 gpurun_out/r05n_ab_k4_$W.txt)   K=8: $(tail -1 gpurun_out/r05n_ab_k8_$W.txt)"
done
