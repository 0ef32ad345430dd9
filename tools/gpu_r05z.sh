#!/bin/bash
# r05: what the drop-in's first frame trace does beyond the steady one (HIP API + kernel trace of two
# timed 'r' presses at the reference's defaults).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05z; export TMPDIR=/tmp
g++ -std=c++17 -O2 -ffp-contract=off -Iinclude tests/cxx/dropin_main.cpp -Lraytracert_amd -lrtamd -Wl,-rpath,$PWD/raytracert_amd -o /tmp/dropin_main || exit 1
python3 -c "import bench, tempfile; print(bench.workload_scene('ref:dodgeColorTest.obj', '/tmp'))" > /tmp/objpath.txt || exit 1
OBJ=$(tail -1 /tmp/objpath.txt)
timeout -k 10 120 /tmp/dropin_main keys $OBJ 500 500 /tmp/f T T T > gpurun_out/r05z/plain.txt 2>&1 || exit 1
grep "^frame" gpurun_out/r05z/plain.txt
