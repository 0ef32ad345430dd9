set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_r03h.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_r03h.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r03h.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
