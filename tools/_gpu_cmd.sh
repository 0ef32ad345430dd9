set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
{ bash tools/ab_bench.sh 3; bash tools/ab_bench.sh 2 --workload c3; bash tools/ab_bench.sh 1 --workload c5 --steps 10; } > gpurun_out/ab_block3.txt 2>&1; cat gpurun_out/ab_block3.txt
