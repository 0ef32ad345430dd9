#!/bin/bash
# Register use, spill and scratch of the chain kernels as hipcc compiles them (device pass only,
# -Rpass-analysis=kernel-resource-usage). Usage: tools/kernel_resources.sh [rt_kernels.hip] [filter]
# The default filter is the C4 timed kernel k_chain<4, true, false, true, false>.
set -euo pipefail
HERE="$(cd "$(dirname "$0")/.." && pwd)"
SRC="${1:-$HERE/raytracert_amd/csrc/rt_kernels.hip}"
FILTER="${2:-k_chainILi4ELb1ELb0ELb1ELb0E}"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
    -I"$HERE/include" -I"$(dirname "$SRC")" -I"$HERE/raytracert_amd/build" ${EXTRA_FLAGS:-} -c "$SRC" -o /tmp/kres_$$.o \
    --offload-device-only -Rpass-analysis=kernel-resource-usage 2>&1 |
    awk -v f="$FILTER" '/Function Name:/ {show = index($0, f) > 0; if (show) print $(NF-1)} show && /VGPRs:|Scratch|Spill|Occupancy/ {sub(/.*remark: +/, ""); sub(/ \[-Rpass.*/, ""); print "   " $0}'
rm -f /tmp/kres_$$.o
