set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cd_tests.log 2>&1 || { tail -30 gpurun_out/cd_tests.log; exit 1; }
tail -1 gpurun_out/cd_tests.log
for L in w6 w5; do echo "== $L"; AB_REF='{"chain_kernel":0}' RTAMD_LIB=$PWD/raytracert_amd/ab/lib_$L.so timeout -k 10 300 python tools/ab_tune.py '[{"chain_kernel":0,"pipes":2},{"chain_kernel":2,"pipes":2},{"chain_kernel":0,"pipes":1},{"chain_kernel":2,"pipes":1}]' 7 2>&1 | grep variant | cut -c1-150 || exit 1; done
AB_REF='{"chain_kernel":0}' timeout -k 10 300 python tools/ab_tune.py '[{"chain_kernel":0,"pipes":2},{"chain_kernel":2,"pipes":2}]' 5 C5 2>&1 | grep variant | cut -c1-150
