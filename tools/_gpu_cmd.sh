set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r03b.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r03b.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r03b.log
for w in c4 c5; do
timeout -k 10 300 python bench.py --workload $w --no-cpu --no-bf-roofline > gpurun_out/bench_r03b_$w.json 2> gpurun_out/bench_r03b_$w.err || { tail -20 gpurun_out/bench_r03b_$w.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r03b_$w.json')); print('$w', d['value'], d['ms_per_step'], 'cold', d['config']['first_frame_ms'], d['config'].get('first_frame_screen_order_ms'), d.get('batches'))"
done
