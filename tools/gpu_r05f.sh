#!/bin/bash
# r05 final: the GPU suite, the default bench line and the reference-defaults line on the final build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r05f_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r05f_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05f_pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/r05f_bench.json 2> gpurun_out/r05f_bench.err || { tail -30 gpurun_out/r05f_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05f_bench.json')); c=d['config']; r=d['roofline']
print('value', d['value'], 'ms', d['ms_per_step'], 'one', c['one_in_flight']['ms_per_step'], 'inflight', c['in_flight']['ms_per_step'], 'first', c['first_frame_ms'], 'orbit', c['orbit']['ms_per_step'], c['orbit']['one_in_flight']['ms_per_step'], c['orbit']['views_per_call']['ms_per_step'])
print('roof', r['frac'], r['avg_launch_ms'], r['rocprof']['mean_us'], r['rocprof']['source'], 'cpu parity', d['cpu_baseline']['parity_vs_gpu']['exact_frac'])"
timeout -k 10 600 python bench.py --workload ref_default --no-bf-roofline > gpurun_out/r05f_bench_ref_default.json 2> gpurun_out/r05f_bench_ref_default.err || { tail -20 gpurun_out/r05f_bench_ref_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05f_bench_ref_default.json')); dl=d['dropin_loop']
print('ref_default', d['value'], d['ms_per_step'], {k: dl[k] for k in ('loop_ms', 'first_loop_ms', 'frame_trace_ms', 'first_frame_trace_ms', 'host_floor_ms')})"
