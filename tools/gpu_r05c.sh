#!/bin/bash
# r05: quad-walk parity + A/B on C4, the new GPU tests, one bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "quad_walk" -m gpu > gpurun_out/r05c_pytest_quad.log 2>&1 || { tail -40 gpurun_out/r05c_pytest_quad.log; exit 1; }
tail -2 gpurun_out/r05c_pytest_quad.log
timeout -k 10 600 python -u tools/ab_frame.py c4 '[{}, {"steal_quarter": 64, "quad_walk": 1}, {"steal_quarter": 256, "quad_walk": 1}, {"steal_quarter": 512, "quad_walk": 1, "steal_half": 0}, {"steal_quarter": 1024, "quad_walk": 1, "steal_half": 0}, {"steal_quarter": 256}]' 3 40 2>&1 | grep -v amdgpu.ids > gpurun_out/r05c_ab_quad_c4.txt || { cat gpurun_out/r05c_ab_quad_c4.txt; exit 1; }
cat gpurun_out/r05c_ab_quad_c4.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernargs.py tests/test_gpu_orbit.py tests/test_gpu_inflight.py tests/test_cxx_dropin.py -m gpu > gpurun_out/r05c_pytest.log 2>&1 || { tail -40 gpurun_out/r05c_pytest.log; exit 1; }
tail -2 gpurun_out/r05c_pytest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-bf-roofline > gpurun_out/r05c_bench.json 2> gpurun_out/r05c_bench.err || { tail -30 gpurun_out/r05c_bench.err; exit 1; }
cat gpurun_out/r05c_bench.json
for lib in "" raytracert_amd/ab/lib_rec0.so "" raytracert_amd/ab/lib_rec0.so; do
  env ${lib:+RTAMD_LIB=$lib} timeout -k 10 300 python -u tools/ab_frame.py c4 '[{}]' 2 40 2>&1 | grep -v amdgpu.ids | sed "s|^|[${lib:-default}] |" >> gpurun_out/r05c_ab_ldsrec.txt || exit 1
done
cat gpurun_out/r05c_ab_ldsrec.txt
