set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/lat" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/latency_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/lat.log" 2>&1
cd "$GRAFT_REPO_ROOT"; grep kind gpurun_out/lat.log
python3 - <<'P'
import csv, glob
f = glob.glob("gpurun_out/lat/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "intersect_only" in r["Kernel_Name"]]
for r in rows:
    print(r["Kernel_Name"][:45], r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size",""), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
P
