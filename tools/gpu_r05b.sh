#!/bin/bash
# r05: new GPU tests (kernarg probe, NaN corners, orbit, dedicated streams, drop-in), a bench line,
# and the in-flight hardware-queue A/B with rt_stream_create streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernargs.py tests/test_gpu_orbit.py tests/test_gpu_inflight.py tests/test_cxx_dropin.py -m gpu > gpurun_out/r05b_pytest.log 2>&1 || { tail -40 gpurun_out/r05b_pytest.log; exit 1; }
tail -3 gpurun_out/r05b_pytest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r05b_bench.json 2> gpurun_out/r05b_bench.err || { tail -30 gpurun_out/r05b_bench.err; exit 1; }
cat gpurun_out/r05b_bench.json
timeout -k 10 600 python bench.py --workload ref_default --steps 20 --warmup 5 --no-cpu > gpurun_out/r05b_bench_ref.json 2> gpurun_out/r05b_bench_ref.err || { tail -30 gpurun_out/r05b_bench_ref.err; exit 1; }
timeout -k 10 600 python tools/ab_inflight2.py ref_default 40 10 "" "rtstreams=1" "" "rtstreams=1" 2>&1 | grep -v amdgpu.ids > gpurun_out/r05b_ab_rtstreams.txt || exit 1
timeout -k 10 600 python tools/ab_inflight2.py c4 40 10 "" "rtstreams=1" 2>&1 | grep -v amdgpu.ids >> gpurun_out/r05b_ab_rtstreams.txt || exit 1
cut -c1-110 gpurun_out/r05b_ab_rtstreams.txt
