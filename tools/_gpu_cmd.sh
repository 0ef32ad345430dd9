set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_cold.py ref_default 6 "" "steal_quarter=64" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_q2.txt || exit 1
timeout -k 10 300 python tools/ab_cold.py c4 4 "" "steal_quarter=64" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_q2.txt || exit 1
timeout -k 10 300 python tools/ab_cold.py c2 4 "" "steal_quarter=64" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_q2.txt || exit 1
timeout -k 10 300 python tools/ab_cold.py c3 4 "" "steal_quarter=64" 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_q2.txt || exit 1
