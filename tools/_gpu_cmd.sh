set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_noslp.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_noslp.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_noslp.log
bash tools/ab_bench.sh 3 2>&1 | tee gpurun_out/ab_sched.txt || exit 1
bash tools/ab_bench.sh 1 --workload c5 --steps 10 2>&1 | tee -a gpurun_out/ab_sched.txt || exit 1
