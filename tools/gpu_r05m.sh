#!/bin/bash
# r05: multi-frame launches with deep chains (records per frame in the workspace): parity, then the
# reference's defaults bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiframe.py tests/test_gpu_orbit.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05m_pytest.log 2>&1 || { tail -30 gpurun_out/r05m_pytest.log; exit 1; }
tail -2 gpurun_out/r05m_pytest.log
timeout -k 10 600 python bench.py --workload ref_default --no-bf-roofline > gpurun_out/r05m_bench_ref_default.json 2> gpurun_out/r05m_bench_ref_default.err || { tail -20 gpurun_out/r05m_bench_ref_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r05m_bench_ref_default.json')); c=d['config']; print(d['value'], d['ms_per_step'], c['value_mode'], 'one', c['one_in_flight']['ms_per_step'], 'inflight', c['in_flight']['ms_per_step'], 'multi', c['multi_frame'], 'dropin', {k: v for k, v in (c.get('dropin_loop') or {}).items() if 'ms' in k}, d['cpu_baseline']['parity_vs_gpu'])"
