set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/coop_tests.log 2>&1 || { tail -30 gpurun_out/coop_tests.log; exit 1; }
tail -1 gpurun_out/coop_tests.log
for pass in 1 2; do for L in co0 co1; do echo "== $L"; RTAMD_LIB=$PWD/raytracert_amd/ab/lib_$L.so timeout -k 10 300 python tools/ab_tune.py '[{}]' 9 2>&1 | grep variant | cut -c1-150 || exit 1; done; done
for L in co0 co1; do echo "== $L C5"; RTAMD_LIB=$PWD/raytracert_amd/ab/lib_$L.so timeout -k 10 300 python tools/ab_tune.py '[{}]' 5 C5 2>&1 | grep variant | cut -c1-150 || exit 1; done
