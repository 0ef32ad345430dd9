#!/bin/bash
# first GPU bring-up: smoke, gpu tests, short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocminfo 2>/dev/null | grep -m3 -E "gfx|Marketing" > gpurun_out/rocminfo.txt || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
exit $rc
