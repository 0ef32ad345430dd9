#!/bin/bash
# Quick GPU session: the GPU tests (one process, per-test time limit) and short bench lines for C4
# and C2. Every GPU step time-limited; stops at the first failure. Usage: tools/gpu_check.sh TAG [pytest-args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "$@" > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --steps 40 --no-cpu --no-bf-roofline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'], d['config'].get('first_frame_ms'))"
timeout -k 10 300 python bench.py --workload c2 --steps 40 --no-cpu --no-bf-roofline > gpurun_out/bench_${TAG}_c2.json 2> gpurun_out/bench_${TAG}_c2.err || { echo "bench c2 failed"; tail -30 gpurun_out/bench_${TAG}_c2.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_${TAG}_c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'], d['config'].get('first_frame_ms'))"
