#!/bin/bash
# Bench lines for the non-default BASELINE configs. C2: the CPU baseline renders the whole frame;
# C3: every 16th tile; C5: every 1024th tile, each with its in-run parity check.
# C5 stochastic is parity-tested in tests/test_gpu_configs.py and runs without the CPU leg here.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02}
for W in ref_default c2 c3 c5 c5s; do
  EXTRA="--no-bf-roofline"
  [ "$W" = "c5s" ] && EXTRA="$EXTRA --no-cpu"
  timeout -k 10 900 python bench.py --workload $W $EXTRA > gpurun_out/bench_${TAG}_$W.json 2> gpurun_out/bench_${TAG}_$W.err || { echo "bench $W failed"; tail -20 gpurun_out/bench_${TAG}_$W.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_$W.json')); c=d.get('cpu_baseline') or {}; print('$W', d['value'], 'Mrays/s', d['ms_per_step'], 'ms', 'cold', d['config']['first_frame_ms'], d['config']['rays_per_step'], 'rays', 'load', d['config']['scene_load_s'], 'cpu', c.get('value'), c.get('parity_vs_gpu'))"
done
