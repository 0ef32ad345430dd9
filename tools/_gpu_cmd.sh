set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -q -k "steal or assemble or shard or sharded" --timeout 120 --timeout-method thread > gpurun_out/pytest_steal.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_steal.log; exit 1; }
tail -1 gpurun_out/pytest_steal.log
TAG=r02f
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" --selected-regions -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 5 --prof-timed-only --no-cpu --no-cold --no-path-compare --no-bf-roofline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1) || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/kernel_trace_summary.py gpurun_out/prof/$TAG 3 > gpurun_out/${TAG}_kernel_trace_summary.json || exit 1
cat gpurun_out/${TAG}_kernel_trace_summary.json | head -c 1500
bash tools/ab_steal_split.sh 2 > gpurun_out/ab_steal_split.txt 2>&1; cat gpurun_out/ab_steal_split.txt
