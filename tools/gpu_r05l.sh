#!/bin/bash
# r05: node-visit build variants under the multi-frame launch, then the other workloads' bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r05k.sh || exit 1
bash tools/gpu_workloads.sh r05j
