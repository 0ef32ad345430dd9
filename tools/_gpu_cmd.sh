set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "shadow_helpers or split_batches or auto or steal or trial or batch_order or cold" > gpurun_out/t_def.log 2>&1 || { tail -30 gpurun_out/t_def.log; exit 1; }
tail -1 gpurun_out/t_def.log
for w in c4 c3 c5 c2 ref_default; do
timeout -k 10 300 python bench.py --workload $w --no-cpu --no-bf-roofline --no-dropin > gpurun_out/bench_h_$w.json 2> gpurun_out/bench_h_$w.err || { tail -20 gpurun_out/bench_h_$w.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_h_$w.json')); c=d['config']; print('$w', d['value'], d['ms_per_step'], 'cold', c['first_frame_ms'], c.get('launch_trials'), d['batches']['max_us'])"
done
