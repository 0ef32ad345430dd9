set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/oe_tests.log 2>&1 || { tail -30 gpurun_out/oe_tests.log; exit 1; }
tail -1 gpurun_out/oe_tests.log
for T in 1 8 1 8; do timeout -k 10 300 python bench.py --no-bf-roofline --no-cpu --tune order_every=$T > gpurun_out/bench_oe.json 2> gpurun_out/bench_oe.err || { tail -20 gpurun_out/bench_oe.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_oe.json')); print('order_every $T', d['value'], d['ms_per_step'])"; done
