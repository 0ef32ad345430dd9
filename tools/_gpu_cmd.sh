set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r02g.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r02g.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r02g.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --no-bf-roofline > gpurun_out/bench_selfreset.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/bench_selfreset.json')); print('frame', d['ms_per_step'], 'chain', d['kernel_ms_per_step'], 'shard_path', d['shard_path']['ms_per_step'], 'cold', d['config']['first_frame_ms'])" || exit 1
done
