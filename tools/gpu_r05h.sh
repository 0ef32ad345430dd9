#!/bin/bash
# r05: default bench line (multi-frame headline), orbit dilation radius A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r05h_bench.json 2> gpurun_out/r05h_bench.err || { tail -30 gpurun_out/r05h_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05h_bench.json')); c=d['config']
print('value', d['value'], 'ms', d['ms_per_step'], c['value_mode'], 'one', c['one_in_flight']['ms_per_step'], 'inflight', c['in_flight']['ms_per_step'], 'first', c['first_frame_ms'])
print('orbit', c['orbit']['ms_per_step'], c['orbit']['one_in_flight'], c['orbit'].get('parity_vs_cpu'))
print('roofline', {k: d['roofline'][k] for k in ('achieved', 'frac', 'avg_launch_ms', 'frames_per_launch')})
print('batches', d['batches']['max_us'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['parity_vs_gpu'])
print('bf', d['roofline_bruteforce'])"
for r in 1 2 3 0 1 2 3; do
  timeout -k 10 600 python -u bench.py --steps 40 --warmup 5 --no-bf-roofline --no-cpu --no-cold --no-path-compare --no-multi-frame --frames-per-call 1 --tune motion_order=$r > gpurun_out/r05h_orbit_r$r.json 2> gpurun_out/r05h_orbit_r$r.err || { tail -30 gpurun_out/r05h_orbit_r$r.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r05h_orbit_r$r.json')); c=d['config']
print('motion_order $r: static', d['ms_per_step'], c['one_in_flight']['ms_per_step'], 'orbit', c['orbit']['ms_per_step'], c['orbit']['one_in_flight']['ms_per_step'])" | tee -a gpurun_out/r05h_orbit_ab.txt
done
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_multi.py c4 '[{}, {"inflight_dynamic": 2}, {"chain_split": 4}, {"chain_split": 0}]' 3 40 4 > gpurun_out/r05i_ab_multi_c4.txt 2>&1 || { tail -30 gpurun_out/r05i_ab_multi_c4.txt; exit 1; }
tail -6 gpurun_out/r05i_ab_multi_c4.txt
