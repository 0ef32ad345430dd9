#!/bin/bash
# r05: the per-piece un-permute and steps per call at N > 1: sharded tests, then the probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05s_pytest.log 2>&1 || { tail -30 gpurun_out/r05s_pytest.log; exit 1; }
tail -2 gpurun_out/r05s_pytest.log
timeout -k 10 300 python -u tools/shard_probe.py 2 4 8 > gpurun_out/r05s_shard_probe.txt 2>&1 || { tail -20 gpurun_out/r05s_shard_probe.txt; exit 1; }
grep "^N" gpurun_out/r05s_shard_probe.txt
