#!/bin/bash
# r05: what the drop-in's first frame trace does beyond the steady one (HIP API + kernel trace of two
# timed 'r' presses at the reference's defaults).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05y; export TMPDIR=/tmp
g++ -std=c++17 -O2 -ffp-contract=off -Iinclude tests/cxx/dropin_main.cpp -Lraytracert_amd -lrtamd -Wl,-rpath,$PWD/raytracert_amd -o /tmp/dropin_main || exit 1
python3 -c "import bench, tempfile; print(bench.workload_scene('ref:dodgeColorTest.obj', '/tmp'))" > /tmp/objpath.txt || exit 1
OBJ=$(tail -1 /tmp/objpath.txt)
timeout -k 10 120 /tmp/dropin_main keys $OBJ 500 500 /tmp/f T T T > gpurun_out/r05y/plain.txt 2>&1 || exit 1
grep "^frame" gpurun_out/r05y/plain.txt
cd /tmp && timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05y/prof -o run -- /tmp/dropin_main keys $OBJ 500 500 /tmp/g T T > $GRAFT_REPO_ROOT/gpurun_out/r05y/prof.txt 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r05y/prof.txt; exit 1; }
grep "^frame" $GRAFT_REPO_ROOT/gpurun_out/r05y/prof.txt
ls -R $GRAFT_REPO_ROOT/gpurun_out/r05y/prof | head
