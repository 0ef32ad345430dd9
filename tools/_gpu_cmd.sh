set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
TAG=r02f
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 500 --warmup 5 --no-cpu --no-cold --no-path-compare --no-bf-roofline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1) || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/kernel_trace_summary.py gpurun_out/prof/$TAG 8 > gpurun_out/${TAG}_kernel_trace_summary.json || exit 1
head -c 1200 gpurun_out/${TAG}_kernel_trace_summary.json
timeout -k 10 300 python bench.py --no-cpu --no-bf-roofline > gpurun_out/bench_shard.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/bench_shard.json')); print('frame', d['ms_per_step'], 'shard_path', d['shard_path'])"
bash tools/ab_steal_split.sh 2 > gpurun_out/ab_steal_split.txt 2>&1; cat gpurun_out/ab_steal_split.txt
