set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dir_tests.log 2>&1 || { tail -30 gpurun_out/dir_tests.log; exit 1; }
tail -1 gpurun_out/dir_tests.log
timeout -k 10 300 python bench.py --no-bf-roofline > gpurun_out/bench_dir.json 2> gpurun_out/bench_dir.err || { tail -20 gpurun_out/bench_dir.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_dir.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['parity_vs_gpu'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/prof/gdir" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 2 --no-cpu --no-bf-roofline --profile-steps 1 > "$GRAFT_REPO_ROOT/gpurun_out/gdir.log" 2>&1) || { tail -5 gpurun_out/gdir.log; exit 1; }
python3 tools/frame_gaps.py $(find gpurun_out/prof/gdir -name "*kernel_trace.csv") 6
