set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/ab_bench.sh 2 > gpurun_out/ab_float_c4.txt 2>&1 || { echo "ab failed"; cat gpurun_out/ab_float_c4.txt; exit 1; }
cat gpurun_out/ab_float_c4.txt
bash tools/ab_bench.sh 1 --workload c2 > gpurun_out/ab_float_c2.txt 2>&1 || { echo "ab c2 failed"; cat gpurun_out/ab_float_c2.txt; exit 1; }
cat gpurun_out/ab_float_c2.txt
bash tools/ab_bench.sh 1 --workload c5 --steps 10 > gpurun_out/ab_float_c5.txt 2>&1 || { echo "ab c5 failed"; cat gpurun_out/ab_float_c5.txt; exit 1; }
cat gpurun_out/ab_float_c5.txt
