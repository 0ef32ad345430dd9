#!/bin/bash
# r05 diagnostics: CU-mask behaviour, C4 batch-lifetime distribution, longest batches alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./build/cumask_probe > gpurun_out/r05a_cumask.txt 2>&1 || { cat gpurun_out/r05a_cumask.txt; exit 1; }
cat gpurun_out/r05a_cumask.txt
timeout -k 10 300 python tools/batch_hist.py c4 40 2>&1 | grep -v amdgpu.ids > gpurun_out/r05a_hist_c4.txt || { cat gpurun_out/r05a_hist_c4.txt; exit 1; }
cat gpurun_out/r05a_hist_c4.txt
timeout -k 10 300 python tools/critical_path.py c4 10 2>&1 | grep -v amdgpu.ids > gpurun_out/r05a_crit_c4.txt || { cat gpurun_out/r05a_crit_c4.txt; exit 1; }
cat gpurun_out/r05a_crit_c4.txt
