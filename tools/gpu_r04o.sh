#!/bin/bash
# r04: RT_OPAQUE_ARGS A/B (raytracert_amd/ab builds a_base, b_opaque): parity of the opaque build,
# bench A/B on C4 / C5 / C2, PMC (instructions, WRITE_SIZE, FETCH_SIZE) of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RTAMD_LIB="$PWD/raytracert_amd/ab/lib_b_opaque.so" timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_lights_samples.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_r04o.log 2>&1 || { tail -30 gpurun_out/pytest_r04o.log; exit 1; }
tail -1 gpurun_out/pytest_r04o.log
bash tools/ab_bench.sh 3 > gpurun_out/ab_r04o.txt 2>&1 || { cat gpurun_out/ab_r04o.txt; exit 1; }
bash tools/ab_bench.sh 2 --workload c5 >> gpurun_out/ab_r04o.txt 2>&1 || { cat gpurun_out/ab_r04o.txt; exit 1; }
bash tools/ab_bench.sh 2 --workload c2 >> gpurun_out/ab_r04o.txt 2>&1 || { cat gpurun_out/ab_r04o.txt; exit 1; }
cat gpurun_out/ab_r04o.txt
PMC_OUT=pmc_o1 bash tools/pmc_ab.sh || exit 1
PMC_OUT=pmc_o2 bash tools/pmc_ab.sh WRITE_SIZE || exit 1
PMC_OUT=pmc_o3 bash tools/pmc_ab.sh FETCH_SIZE || exit 1
for d in pmc_o1 pmc_o2 pmc_o3; do python3 tools/pmc_ab_summary.py gpurun_out/$d; done > gpurun_out/pmc_r04o.txt
cat gpurun_out/pmc_r04o.txt
