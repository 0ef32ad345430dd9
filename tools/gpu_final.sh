#!/bin/bash
# Round evidence in one GPU call: parity tests, PMC passes of the bench's chain kernel (summary
# also placed in profiles/ so the bench line's `traffic` uses it), the default bench line, its
# rocprofv3 kernel stats + per-launch trace summary, and the other BASELINE workloads. Every step
# time-limited; stops at the first failure. Usage: tools/gpu_final.sh TAG [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu_$TAG.log
fi
bash tools/gpu_pmc.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc/$TAG gpurun_out/${TAG}_pmc.json > /dev/null && cp gpurun_out/${TAG}_pmc.json profiles/${TAG}_pmc.json
# the same passes over the 1M-triangle workload (bench --workload c5 reads profiles/*_pmc_c5.json)
WORKLOAD=c5 bash tools/gpu_pmc.sh ${TAG}_c5 > gpurun_out/pmc_${TAG}_c5.log 2>&1 || { echo "pmc c5 failed"; tail -20 gpurun_out/pmc_${TAG}_c5.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc/${TAG}_c5 gpurun_out/${TAG}_pmc_c5.json > /dev/null && cp gpurun_out/${TAG}_pmc_c5.json profiles/${TAG}_pmc_c5.json
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
# rocprof of the timed entry point: 50 ordered frames dilute the first (unordered) launches; the
# trace summary also gives the mean over launches after the first 3
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 500 --warmup 30 --inflight 1 --no-cpu --no-cold --no-path-compare --no-bf-roofline --orbit-step 0 --no-multi-frame --profile-steps 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1) || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python3 tools/kernel_trace_summary.py gpurun_out/prof/$TAG 3 > gpurun_out/${TAG}_kernel_trace_summary.json || exit 1
[ -n "$NO_WORKLOADS" ] || bash tools/gpu_workloads.sh $TAG || exit 1
