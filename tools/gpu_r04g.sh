#!/bin/bash
# r04: parity of the packed node test first (fail fast), then A/B of the builds in raytracert_amd/ab
# on C4 (one frame in flight and the headline mode) and C2. Usage: tools/gpu_r04g.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04g}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_parity_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_parity_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_parity_$TAG.log
bash tools/ab_bench.sh 2 > gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
bash tools/ab_bench.sh 2 --workload c2 >> gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
bash tools/ab_bench.sh 1 --workload ref_default >> gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
