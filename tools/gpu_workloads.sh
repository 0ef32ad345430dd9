#!/bin/bash
# Bench lines for the non-default BASELINE configs (no CPU baseline: C5's brute-force CPU cost is hours).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r01}
for W in c2 c3 c5 c5s; do
  timeout -k 10 500 python bench.py --workload $W --no-cpu --no-bf-roofline > gpurun_out/bench_${TAG}_$W.json 2> gpurun_out/bench_${TAG}_$W.err || { echo "bench $W failed"; tail -20 gpurun_out/bench_${TAG}_$W.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_$W.json')); print('$W', d['value'], 'Mrays/s', d['ms_per_step'], 'ms', d['config']['rays_per_step'], 'rays', 'load', d['config']['scene_load_s'], 'gen', d['config']['scene_gen_s'], d['kernel_ms_per_step'], d['accel'])"
done
