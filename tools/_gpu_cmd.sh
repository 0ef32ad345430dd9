set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "cold or auto or knobs" > gpurun_out/t_auto.log 2>&1 || { tail -30 gpurun_out/t_auto.log; exit 1; }
tail -2 gpurun_out/t_auto.log
for w in c4 c5 c3; do
timeout -k 10 300 python bench.py --workload $w --no-cpu --no-bf-roofline > gpurun_out/bench_r03d_$w.json 2> gpurun_out/bench_r03d_$w.err || { tail -20 gpurun_out/bench_r03d_$w.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r03d_$w.json')); c=d['config']; print('$w', d['value'], d['ms_per_step'], 'cold', c['first_frame_ms'], c.get('first_frame_screen_order_ms'), c.get('launch_trials'))"
done
