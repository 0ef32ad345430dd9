#!/bin/bash
# r04: RT_OPAQUE_ARGS 1 vs 2 A/B (raytracert_amd/ab builds b_opaque1, c_opaque2): parity of 2, bench A/B, PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RTAMD_LIB="$PWD/raytracert_amd/ab/lib_c_opaque2.so" timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_lights_samples.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r04o2.log 2>&1 || { tail -30 gpurun_out/pytest_r04o2.log; exit 1; }
tail -1 gpurun_out/pytest_r04o2.log
bash tools/ab_bench.sh 3 > gpurun_out/ab_r04o2.txt 2>&1 || { cat gpurun_out/ab_r04o2.txt; exit 1; }
bash tools/ab_bench.sh 2 --workload c5 >> gpurun_out/ab_r04o2.txt 2>&1 || { cat gpurun_out/ab_r04o2.txt; exit 1; }
bash tools/ab_bench.sh 1 --workload ref_default --no-dropin >> gpurun_out/ab_r04o2.txt 2>&1 || { cat gpurun_out/ab_r04o2.txt; exit 1; }
cat gpurun_out/ab_r04o2.txt
PMC_OUT=pmc_p1 bash tools/pmc_ab.sh || exit 1
PMC_OUT=pmc_p2 bash tools/pmc_ab.sh WRITE_SIZE || exit 1
for d in pmc_p1 pmc_p2; do python3 tools/pmc_ab_summary.py gpurun_out/$d; done > gpurun_out/pmc_r04o2.txt
cat gpurun_out/pmc_r04o2.txt
