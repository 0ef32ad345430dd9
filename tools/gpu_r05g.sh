#!/bin/bash
# r05: orbit with and without the motion-aware order; orbit/multi-frame parity; bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_orbit.py tests/test_gpu_multiframe.py -m gpu > gpurun_out/r05g_pytest.log 2>&1 || { tail -30 gpurun_out/r05g_pytest.log; exit 1; }
tail -2 gpurun_out/r05g_pytest.log
for v in 1 0 1 0; do
  timeout -k 10 600 python -u bench.py --steps 40 --warmup 5 --no-bf-roofline --no-cpu --no-cold --no-path-compare --no-multi-frame --tune motion_order=$v > gpurun_out/r05g_bench_m$v.json 2> gpurun_out/r05g_bench_m$v.err || { tail -30 gpurun_out/r05g_bench_m$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r05g_bench_m$v.json')); c=d['config']
print('motion_order $v: static', d['ms_per_step'], c['one_in_flight']['ms_per_step'], 'orbit', c['orbit']['ms_per_step'], c['orbit']['one_in_flight']['ms_per_step'], c['orbit'].get('parity_vs_cpu'))" | tee -a gpurun_out/r05g_orbit_ab.txt
done
