set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ord_tests.log 2>&1 || { tail -30 gpurun_out/ord_tests.log; exit 1; }
tail -1 gpurun_out/ord_tests.log
AB_REF='{"batch_order":0}' timeout -k 10 300 python tools/ab_tune.py '[{"batch_order":0},{"batch_order":1}]' 9 2>&1 | grep variant | cut -c1-150
AB_REF='{"batch_order":0}' timeout -k 10 300 python tools/ab_tune.py '[{"batch_order":0},{"batch_order":1}]' 5 C5 2>&1 | grep variant | cut -c1-150
timeout -k 10 300 python bench.py --no-bf-roofline --no-cpu > gpurun_out/bench_ord.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/bench_ord.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
