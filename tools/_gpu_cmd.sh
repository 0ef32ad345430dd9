set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sc_tests.log 2>&1 || { tail -30 gpurun_out/sc_tests.log; exit 1; }
tail -1 gpurun_out/sc_tests.log
for r in 1 2; do timeout -k 10 300 python bench.py --no-bf-roofline --no-cpu > gpurun_out/bench_sc.json 2> gpurun_out/bench_sc.err || { tail -20 gpurun_out/bench_sc.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_sc.json')); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"; done
