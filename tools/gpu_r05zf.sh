#!/bin/bash
# r05 final (paired shadow helpers): the default bench line (citing this build's PMC and rocprof), the
# driver-args line, and the other workloads.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/r05zf_bench.json 2> gpurun_out/r05zf_bench.err || { tail -30 gpurun_out/r05zf_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05zf_bench.json')); c=d['config']; r=d['roofline']
print('value', d['value'], 'ms', d['ms_per_step'], 'one', c['one_in_flight']['ms_per_step'], 'inflight', c['in_flight']['ms_per_step'], 'first', c['first_frame_ms'], 'orbit', c['orbit']['ms_per_step'], c['orbit']['one_in_flight']['ms_per_step'], c['orbit']['views_per_call']['ms_per_step'])
print('roof', r['frac'], r['avg_launch_ms'], r['rocprof']['mean_us'], r['rocprof']['source'], r['dram']['source'], 'cpu parity', d['cpu_baseline']['parity_vs_gpu']['exact_frac'])"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05zf_bench_driver_args.json 2>/dev/null || exit 1
bash tools/gpu_workloads.sh r05zf
