#!/bin/bash
# r04: in-flight own-stream parity + A/B, then BVH build-parameter A/B (raytracert_amd/ab builds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflight.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r04w.log 2>&1 || { tail -20 gpurun_out/pytest_r04w.log; exit 1; }
tail -1 gpurun_out/pytest_r04w.log
timeout -k 10 400 python tools/ab_inflight2.py ref_default 40 10 "" "inflight_streams=1" "" "inflight_streams=1" "" "inflight_streams=1" 2>/dev/null | cut -c1-120 > gpurun_out/ab_r04w.txt || exit 1
timeout -k 10 300 python tools/ab_inflight2.py c4 60 10 "" "inflight_streams=1" "" "inflight_streams=1" 2>/dev/null | cut -c1-120 >> gpurun_out/ab_r04w.txt || exit 1
cat gpurun_out/ab_r04w.txt
bash tools/ab_bench.sh 2 > gpurun_out/ab_r04x.txt 2>&1 || { cat gpurun_out/ab_r04x.txt; exit 1; }
bash tools/ab_bench.sh 2 --workload c2 >> gpurun_out/ab_r04x.txt 2>&1 || { cat gpurun_out/ab_r04x.txt; exit 1; }
bash tools/ab_bench.sh 1 --workload ref_default --no-dropin >> gpurun_out/ab_r04x.txt 2>&1 || { cat gpurun_out/ab_r04x.txt; exit 1; }
cat gpurun_out/ab_r04x.txt
