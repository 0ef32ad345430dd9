set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in c4 c3 c2 c5; do
timeout -k 10 300 python tools/ab_inflight.py $w 1 2 3 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_inflight.txt || exit 1
done
