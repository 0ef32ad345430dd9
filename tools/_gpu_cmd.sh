set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fu_tests.log 2>&1 || { tail -30 gpurun_out/fu_tests.log; exit 1; }
tail -1 gpurun_out/fu_tests.log
for T in 0 1 0 1; do timeout -k 10 300 python bench.py --no-bf-roofline --no-cpu --tune fuse_pixels=$T > gpurun_out/bench_fu.json 2> gpurun_out/bench_fu.err || { tail -20 gpurun_out/bench_fu.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_fu.json')); print('fuse $T', d['value'], d['ms_per_step'])"; done
