#!/bin/bash
# r05: multi-frame launches (parity + bench leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiframe.py tests/test_gpu_kernargs.py -m gpu > gpurun_out/r05f_pytest.log 2>&1 || { tail -30 gpurun_out/r05f_pytest.log; exit 1; }
tail -2 gpurun_out/r05f_pytest.log
timeout -k 10 600 python -u bench.py --steps 40 --warmup 5 --no-bf-roofline --no-cpu > gpurun_out/r05f_bench.json 2> gpurun_out/r05f_bench.err || { tail -30 gpurun_out/r05f_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05f_bench.json')); c=d['config']
print('value', d['value'], 'ms', d['ms_per_step'], 'one', c['one_in_flight']['ms_per_step'], 'first', c['first_frame_ms'])
print('multi', json.dumps(c['multi_frame']))
print('orbit', c['orbit']['ms_per_step'], c['orbit']['one_in_flight'])
print('batches', d['batches']['max_us'])"
timeout -k 10 600 python -u bench.py --workload ref_default --steps 40 --warmup 5 --no-bf-roofline --no-cpu --no-dropin > gpurun_out/r05f_bench_ref.json 2> gpurun_out/r05f_bench_ref.err || { tail -30 gpurun_out/r05f_bench_ref.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r05f_bench_ref.json')); c=d['config']
print('ref value', d['value'], 'ms', d['ms_per_step'], 'one', c['one_in_flight']['ms_per_step'])
print('multi', json.dumps(c['multi_frame']))"
