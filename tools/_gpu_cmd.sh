set -o pipefail
cd "$GRAFT_REPO_ROOT"
AB_REF='{"chain_split":0}' timeout -k 10 400 python tools/ab_tune.py '[{"chain_split":0,"top_nodes":0},{"chain_split":3,"top_nodes":0},{"chain_split":0,"top_nodes":21},{"chain_split":3,"top_nodes":21},{"chain_split":3,"top_nodes":85}]' 5 C5 2>&1 | cut -c1-170
