set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in c4 ref_default c2; do
timeout -k 10 200 python tools/critical_path.py $w 6 > gpurun_out/crit_$w.txt 2>&1 || { echo "crit $w failed"; tail -30 gpurun_out/crit_$w.txt; exit 1; }
cat gpurun_out/crit_$w.txt
done
