#!/bin/bash
# The drop-in's reference-API path at the reference's defaults (dodgeColorTest.obj, 500x500, pf 3,
# max_lvl 10): tests/cxx/dropin_main.cpp built against include/raytracert_dropin.hpp, keys T T R H H
# (two literal 'r' loops, renderImage, the host-floor loop twice), under rocprofv3 --kernel-trace
# --stats, plus the host timers the program prints. Usage: tools/gpu_dropin_profile.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04}
OUT="$GRAFT_REPO_ROOT/gpurun_out/dropin_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "import sys; sys.path.insert(0, 'tests'); from _util import materialize_models; materialize_models('$OUT/models')" || exit 1
g++ -std=c++17 -O2 -ffp-contract=off -Iinclude tests/cxx/dropin_main.cpp -Lraytracert_amd -lrtamd \
    -Wl,-rpath,"$GRAFT_REPO_ROOT/raytracert_amd" -o "$OUT/dropin_main" || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    "$OUT/dropin_main" keys "$OUT/models/dodgeColorTest.obj" 500 500 "$OUT/f" T T R H H > "$OUT/host_timers.txt" 2>&1 || exit 1
grep -E "^frame |^hostfloor " "$OUT/host_timers.txt"
