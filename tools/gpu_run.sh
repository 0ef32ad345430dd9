#!/bin/bash
# The one GPU-call runner (r06; replaces the per-run tools/gpu_r0*.sh scripts, whose command lines are
# kept in profiles/COMMANDS.md). Usage: tools/gpu_run.sh TAG STEP [STEP ...]
# Steps (each time-limited; the script stops at the first failure; outputs under gpurun_out/):
#   tests        pytest -m gpu
#   strong_c4    strong-scaling shares on one GPU, C4 (tools/strong_probe.py; STRONG_VARIANTS, STRONG_LIB)
#   strong_c5    the same for C5
#   phases       per-phase VALU PMC of the four-frame launch (tools/phase_probe.py + tools/phase_summary.py)
#   bench        python bench.py (driver defaults; BENCH_ARGS extra)
#   pmc          tools/gpu_pmc.sh TAG + summary into profiles/TAG_pmc.json
#   rocprof      rocprofv3 --kernel-trace --stats of the bench's timed entry point + trace summary
#   workloads    tools/gpu_workloads.sh TAG (the other BASELINE workloads)
#   e2e          bench.py --e2e-only: render -> host -> PPM per C4 frame
#   ab           same-box A/B of library builds (AB_LIBS: names of raytracert_amd/ab/lib_<name>.so, 'cur' = the
#                in-tree build; AB_PASSES; AB_WORKLOADS; AB_ARGS extra bench arguments): the timed loop only
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }
for STEP in "$@"; do
  case $STEP in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || fail tests gpurun_out/pytest_gpu_$TAG.log
      tail -1 gpurun_out/pytest_gpu_$TAG.log ;;
    strong_c4|strong_c5)
      WL=${STEP#strong_}
      for V in ${STRONG_VARIANTS:-default}; do
        L=""; case $V in lib=*) L=${V%%:*}; L=${L#lib=}; V=${V#*:} ;; esac
        RTAMD_LIB=${L:+raytracert_amd/ab/lib_$L.so} timeout -k 10 300 python -u tools/strong_probe.py $WL ${STRONG_NS:-2,4,8} "$V" \
          >> gpurun_out/strong_${WL}_$TAG.jsonl 2>> gpurun_out/strong_${WL}_$TAG.err || fail $STEP gpurun_out/strong_${WL}_$TAG.err
        [ -n "$L" ] && sed -i "\$s/\"variant\": \"/\"variant\": \"lib=$L:/" gpurun_out/strong_${WL}_$TAG.jsonl
      done
      tail -n 20 gpurun_out/strong_${WL}_$TAG.jsonl ;;
    phases)
      mkdir -p gpurun_out/phase_$TAG
      for V in all no_specular no_shadows no_secondary no_shadows_no_secondary; do
        (cd /tmp && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
          -d "$GRAFT_REPO_ROOT/gpurun_out/phase_$TAG/$V/sq" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/phase_probe.py" $V 20 \
          > "$GRAFT_REPO_ROOT/gpurun_out/phase_$TAG/$V.log" 2>&1) || fail phases gpurun_out/phase_$TAG/$V.log
        grep "ms per frame" gpurun_out/phase_$TAG/$V.log
      done
      python3 tools/phase_summary.py gpurun_out/phase_$TAG gpurun_out/${TAG}_valu_phases.json > gpurun_out/phase_$TAG/summary.txt || fail phase_summary gpurun_out/phase_$TAG/summary.txt
      cat gpurun_out/phase_$TAG/summary.txt | head -80 ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || fail bench gpurun_out/bench_$TAG.err
      cat gpurun_out/bench_$TAG.json ;;
    pmc)
      bash tools/gpu_pmc.sh $TAG > gpurun_out/pmc_$TAG.log 2>&1 || fail pmc gpurun_out/pmc_$TAG.log
      python3 tools/pmc_summary.py gpurun_out/pmc/$TAG gpurun_out/${TAG}_pmc.json > /dev/null || exit 1 ;;
    rocprof)
      mkdir -p gpurun_out/prof
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 500 --warmup 30 --inflight 1 --no-cpu --no-cold --no-path-compare --no-bf-roofline --orbit-step 0 --no-multi-frame --no-strong-shares --no-e2e --no-dropin --profile-steps 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1) || fail rocprof gpurun_out/prof_$TAG.log
      python3 tools/kernel_trace_summary.py gpurun_out/prof/$TAG 3 > gpurun_out/${TAG}_kernel_trace_summary.json || exit 1 ;;
    workloads)
      bash tools/gpu_workloads.sh $TAG || exit 1 ;;
    e2e)
      timeout -k 10 300 python bench.py --e2e-only > gpurun_out/e2e_$TAG.json 2> gpurun_out/e2e_$TAG.err || fail e2e gpurun_out/e2e_$TAG.err
      cat gpurun_out/e2e_$TAG.json ;;
    ab)
      for P in $(seq 1 ${AB_PASSES:-2}); do
        for W in ${AB_WORKLOADS:-c4}; do
          for L in ${AB_LIBS:-cur}; do
            LIBV=""; [ "$L" != "cur" ] && LIBV=raytracert_amd/ab/lib_$L.so
            R=$(RTAMD_LIB=$LIBV timeout -k 10 300 python bench.py --workload $W --no-cpu --no-bf-roofline --no-cold --no-path-compare \
                --no-dropin --no-strong-shares --no-e2e --orbit-step 0 --no-multi-frame ${AB_ARGS:-} 2>gpurun_out/ab_$TAG.err) || fail ab gpurun_out/ab_$TAG.err
            echo "$R" >> gpurun_out/ab_$TAG.jsonl
            echo "$R" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; b=d.get("batches") or {}; print(sys.argv[1], sys.argv[2], "pass", sys.argv[3], d["ms_per_step"], "ms", "one", (c.get("one_in_flight") or {}).get("ms_per_step"), "in_flight", (c.get("in_flight") or {}).get("ms_per_step"), "chain", d["roofline"]["avg_launch_ms"], "batch max", b.get("max_us"))' $W $L $P
          done
        done
      done ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
