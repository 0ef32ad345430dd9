#!/bin/bash
# r04: where the chain kernel's per-batch kernel-argument reads land. Bench (one and two in flight)
# under HIP_FORCE_DEV_KERNARG unset / 1 / 0, then the rocprofv3 kernel trace of the base (arguments
# held from the start) and opaque (read per batch) builds on the same box, against their own events.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kernarg
export TMPDIR=/tmp
B="--no-cpu --no-cold --no-path-compare --no-bf-roofline --steps 100"
S='import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms", d["config"]["one_in_flight"]["ms_per_step"], "one", "events", d["roofline"]["avg_launch_ms"], "chain", d["kernel_ms_per_step"]["chain"])'
for e in unset 1 0; do
  for L in a_base b_opaque1; do
    if [ $e = unset ]; then R=$(RTAMD_LIB="$PWD/raytracert_amd/ab/lib_$L.so" timeout -k 10 200 python bench.py $B 2>/dev/null) || exit 1
    else R=$(HIP_FORCE_DEV_KERNARG=$e RTAMD_LIB="$PWD/raytracert_amd/ab/lib_$L.so" timeout -k 10 200 python bench.py $B 2>/dev/null) || exit 1; fi
    echo "DEV_KERNARG=$e $L $(echo "$R" | python -c "$S")"
  done
done
for L in a_base b_opaque1; do
  (cd /tmp && RTAMD_LIB="$GRAFT_REPO_ROOT/raytracert_amd/ab/lib_$L.so" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/kernarg/$L" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 300 --warmup 30 --inflight 1 --no-cpu --no-cold --no-path-compare --no-bf-roofline > "$GRAFT_REPO_ROOT/gpurun_out/kernarg/$L.json" 2>/dev/null) || exit 1
  echo "rocprof $L line: $(python -c "$S" < gpurun_out/kernarg/$L.json) trace: $(python3 tools/kernel_trace_summary.py gpurun_out/kernarg/$L 3 | python -c 'import json,sys; k=json.load(sys.stdin)["kernels"]["k_chain<4, true, false, true, false>"]; print(k["launches"], "launches mean", k["mean_after_first_3_us"], "median", k["median_us"])')"
done
