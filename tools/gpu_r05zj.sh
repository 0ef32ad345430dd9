#!/bin/bash
# r05 final tree: GPU suite, smoke, the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r05zj_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05zj_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05zj_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r05zj_bench.json 2> gpurun_out/r05zj_bench.err || { tail -20 gpurun_out/r05zj_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r05zj_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('value_mode'))"
