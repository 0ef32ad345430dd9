#!/bin/bash
# r05: a new view's first frame under cold-launch variants (order estimate, distribution, stealing).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/cold_probe.py '[{}, {"cold_estimate": 1}, {"cold_estimate": 0}, {"wave_steal": 1}, {"cold_estimate": 1, "wave_steal": 1}, {"steal_half": 2048}, {"steal_half": 8192, "steal_quarter": 1024}]' 7 > gpurun_out/r05w_cold_probe.txt 2>&1 || { tail -20 gpurun_out/r05w_cold_probe.txt; exit 1; }
cat gpurun_out/r05w_cold_probe.txt | grep round
