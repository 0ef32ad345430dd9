#!/bin/bash
# r05: frames in flight on plain torch streams vs rt_stream_create (CU-masked, own queue) streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_inflight2.py c4 40 10 "" "rtstreams=1" "" "rtstreams=1" > gpurun_out/r05e_ab_rtstreams.txt 2>&1 || { cat gpurun_out/r05e_ab_rtstreams.txt; exit 1; }
timeout -k 10 600 python -u tools/ab_inflight2.py ref_default 40 10 "" "rtstreams=1" >> gpurun_out/r05e_ab_rtstreams.txt 2>&1 || { cat gpurun_out/r05e_ab_rtstreams.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05e_ab_rtstreams.txt | cut -c1-120
