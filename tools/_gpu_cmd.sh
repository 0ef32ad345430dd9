set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_r03h.json 2> gpurun_out/bench_r03h.err || { echo "bench failed"; tail -30 gpurun_out/bench_r03h.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r03h.json')); c=d['config']; print('c4', d['value'], d['ms_per_step'], c['first_frame_ms'], c['one_in_flight'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], (d['cpu_baseline'] or {}).get('parity_vs_gpu'))"
for w in c3 c2 ref_default c5; do
timeout -k 10 300 python bench.py --workload $w --no-bf-roofline --no-dropin > gpurun_out/bench_r03h_$w.json 2> gpurun_out/bench_r03h_$w.err || { tail -20 gpurun_out/bench_r03h_$w.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r03h_$w.json')); c=d['config']; print('$w', d['value'], d['ms_per_step'], c['first_frame_ms'], c['one_in_flight'], (d['cpu_baseline'] or {}).get('parity_vs_gpu'))"
done
