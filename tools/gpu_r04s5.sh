#!/bin/bash
# r04: stealing chain kernel at 4 (default) vs 5 waves per EU (raytracert_amd/ab a_steal4, b_steal5;
# with the kernel arguments read per batch its spill at 5 is 88 B per lane): parity of 5, bench A/B
# on the workloads whose trials pick the stealing kernel (C2, ref_default) and C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RTAMD_LIB="$PWD/raytracert_amd/ab/lib_b_steal5.so" timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r04s5.log 2>&1 || { tail -30 gpurun_out/pytest_r04s5.log; exit 1; }
tail -1 gpurun_out/pytest_r04s5.log
bash tools/ab_bench.sh 3 --workload c2 > gpurun_out/ab_r04s5.txt 2>&1 || { cat gpurun_out/ab_r04s5.txt; exit 1; }
bash tools/ab_bench.sh 2 --workload ref_default --no-dropin >> gpurun_out/ab_r04s5.txt 2>&1 || { cat gpurun_out/ab_r04s5.txt; exit 1; }
bash tools/ab_bench.sh 2 --workload c3 >> gpurun_out/ab_r04s5.txt 2>&1 || { cat gpurun_out/ab_r04s5.txt; exit 1; }
bash tools/ab_bench.sh 1 >> gpurun_out/ab_r04s5.txt 2>&1 || { cat gpurun_out/ab_r04s5.txt; exit 1; }
cat gpurun_out/ab_r04s5.txt
