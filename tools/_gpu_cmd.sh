set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof/r01m_p1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-bf-roofline --pipes 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_r01m_p1.log" 2>&1) || { tail -20 gpurun_out/prof_r01m_p1.log; exit 1; }
grep -h "k_chain" gpurun_out/prof/r01m_p1/run_kernel_stats.csv | cut -c1-60,200-400
tail -1 gpurun_out/prof_r01m_p1.log | cut -c1-300
