#!/bin/bash
# r05: quad instantiation penalty vs tier effect, LDS chain records A/B, FMA drop-in test, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cxx_dropin.py -k "fma" -m gpu > gpurun_out/r05d_pytest_fma.log 2>&1 || { tail -20 gpurun_out/r05d_pytest_fma.log; exit 1; }
tail -2 gpurun_out/r05d_pytest_fma.log
timeout -k 10 600 python -u tools/ab_frame.py c4 '[{}, {"steal_quarter": 1, "quad_walk": 1}, {"steal_quarter": 256, "quad_walk": 1, "steal_half": 256}, {"steal_quarter": 128, "quad_walk": 1}, {"steal_quarter": 64}]' 3 40 > gpurun_out/r05d_ab_quad_c4.txt 2>&1 || { cat gpurun_out/r05d_ab_quad_c4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05d_ab_quad_c4.txt | tail -7
for lib in "" raytracert_amd/ab/lib_rec0.so "" raytracert_amd/ab/lib_rec0.so; do
  env ${lib:+RTAMD_LIB=$lib} timeout -k 10 300 python -u tools/ab_frame.py c4 '[{}]' 2 40 >> gpurun_out/r05d_ab_ldsrec.txt 2>&1 || exit 1
  echo "[${lib:-default}] done" >> gpurun_out/r05d_ab_ldsrec.txt
done
grep -v amdgpu.ids gpurun_out/r05d_ab_ldsrec.txt | grep "summary\|{}\|done" 
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-bf-roofline > gpurun_out/r05d_bench.json 2> gpurun_out/r05d_bench.err || { tail -30 gpurun_out/r05d_bench.err; exit 1; }
cat gpurun_out/r05d_bench.json
