set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r02h.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r02h.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r02h.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02h.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r02h.log; exit 1; }
echo smoke ok
for W in c4 c2; do
timeout -k 10 300 python bench.py --workload $W --no-cpu --no-bf-roofline > gpurun_out/bench_b256_$W.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/bench_b256_$W.json')); print('$W', d['ms_per_step'], d['value'], 'chain', d['kernel_ms_per_step']['chain'], 'shard', d['shard_path']['ms_per_step'] if d.get('shard_path') else None, 'cold', d['config']['first_frame_ms'])" || exit 1
done
