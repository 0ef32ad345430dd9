#!/bin/bash
# C2 latency probe: per-wave lifetimes of the chain launch (diagnostic -DRT_WAVE_TIMES build from
# tools/build_ab.sh wt "-DRT_WAVE_TIMES") for C2 and C4, and a rocprofv3 kernel trace of the C2 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for W in c2 c4; do
  RTAMD_LIB=$GRAFT_REPO_ROOT/raytracert_amd/ab/lib_wt.so WORKLOAD=$W timeout -k 10 120 python tools/wave_times.py > gpurun_out/${TAG}_wave_times_$W.txt 2>&1 || { echo "wave_times $W failed"; tail -5 gpurun_out/${TAG}_wave_times_$W.txt; exit 1; }
  head -4 gpurun_out/${TAG}_wave_times_$W.txt
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof/${TAG}_c2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c2 --steps 30 --warmup 2 --no-cpu --no-cold --no-path-compare --no-bf-roofline > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_c2.log" 2>&1) || { echo "rocprof failed"; tail -20 gpurun_out/prof_${TAG}_c2.log; exit 1; }
python3 tools/kernel_trace_summary.py gpurun_out/prof/${TAG}_c2 3
