#!/bin/bash
# Round-4 GPU session: the GPU tests (one process, per-test time limit; no -x so every failure is
# listed), then the driver's bench command on C4 and the reference-default workload with the drop-in
# loop. Every GPU step time-limited; a failing step ends the script. Usage: tools/gpu_r04.sh TAG [pytest-args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread "$@" > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-bf-roofline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); c=d['config']; print('c4', d['value'], d['ms_per_step'], c['value_mode'], c['one_in_flight'], c['calibration_frames'], c['launch_trials'], d['cpu_baseline']['parity_vs_gpu'])"
timeout -k 10 400 python bench.py --workload ref_default --steps 20 --warmup 5 --no-bf-roofline > gpurun_out/bench_${TAG}_ref.json 2> gpurun_out/bench_${TAG}_ref.err || { echo "bench ref failed"; tail -30 gpurun_out/bench_${TAG}_ref.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}_ref.json').read().strip().splitlines()[-1]); c=d['config']; print('ref', d['value'], d['ms_per_step'], c['value_mode'], c['one_in_flight'], c['launch_trials'], d.get('dropin_loop'), d['cpu_baseline']['parity_vs_gpu'])"
