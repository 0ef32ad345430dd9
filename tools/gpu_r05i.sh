#!/bin/bash
# r05: multi-frame calls, trials' distribution vs dynamic wave tasks (RT_TUNE_INFLIGHT_DYNAMIC 2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_multi.py c4 '[{}, {"inflight_dynamic": 2}, {"chain_split": 4}, {"chain_split": 0}]' 3 40 4 > gpurun_out/r05i_ab_multi_c4.txt 2>&1 || { tail -30 gpurun_out/r05i_ab_multi_c4.txt; exit 1; }
tail -6 gpurun_out/r05i_ab_multi_c4.txt
