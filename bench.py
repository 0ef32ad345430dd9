#!/usr/bin/env python3
"""Benchmark: Mrays/s + wall-clock per frame at 1920x1080 on the ~100k-triangle synthetic OBJ
(BASELINE.json metric; SURVEY.md §8d configuration C4: 8x8 grid of 40x21 UV spheres + back
plane = 102,402 triangles, pf 1, max_lvl 3, lights (0,0,4) and (1.5,1.5,4)).

A step renders one 1920x1080 frame's worth of 16x16 tiles per GPU: the step's batch is N frames
of the same view whose tiles are interleaved over the N ranks (tile g -> rank g mod N), each rank
renders its tiles with librtamd.so into HBM, and rank 0 collects them with one RCCL gather and
un-permutes them on the device (weak scaling: fixed work per GPU). `--mode strong` instead splits
ONE frame over the N ranks. A ray is one intersectMesh-equivalent query (primary + secondary +
shadow), counted on the device.

    python bench.py [--gpus N --steps K --warmup W]          # N>1: under torch.distributed.run

Prints one JSON line on rank 0. See DESIGN.md §Measurement for the roofline and CPU-baseline
definitions.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "Mrays/s + wall-clock per frame at 1920×1080, 100k-tri OBJ"
FLOP_PER_TEST = 37            # fp32 ops of rayIntersectTriangle's dominant path
FLOP_PER_NODE = 52            # BVH node visit: 2 slab tests (6 sub + 6 mul + 12 min/max each) + 2 distance culls
FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 vector (= FP32 matrix) peak
HBM_PEAK_GBS = 8000.0
TILE = 16
# BASELINE.json configs. C4 is the metric's configuration and the default; the
# others are available with --workload (C1 is the reference's own CPU-only plumbing case).
WORKLOADS = {
    "c4": dict(desc="C4: synthetic 8x8 UV-sphere grid OBJ (102,402 tris) 1920x1080, pf 1, depth 3, 2 lights",
               scene="syn:C4", width=1920, height=1080, pf=1, max_lvl=3, lights=((0.0, 0.0, 4.0), (1.5, 1.5, 4.0))),
    "c2": dict(desc="C2: dodgeColorTest.obj (16,311 tris) 800x600, pf 1, depth 1, 1 light",
               scene="ref:dodgeColorTest.obj", width=800, height=600, pf=1, max_lvl=1, lights=((0.0, 0.0, 4.0),)),
    "c3": dict(desc="C3: Balls surrogate (3 UV spheres 48x24 + ground quad, Balls.mtl materials) 1920x1080, pf 1, "
                    "depth 3, 2 lights (Balls.obj is missing from the reference)",
               scene="syn:balls", width=1920, height=1080, pf=1, max_lvl=3, lights=((0.0, 0.0, 4.0), (2.0, 2.0, 4.0))),
    "c5": dict(desc="C5: synthetic 16x16 UV-sphere grid OBJ (1,015,810 tris) 3840x2160, pf 2 (4 samples/pixel, "
                    "the reference's regular AA grid), depth 3, 4 lights",
               scene="syn:C5", width=3840, height=2160, pf=2, max_lvl=3,
               lights=((0.0, 0.0, 4.0), (1.5, 1.5, 4.0), (-1.5, 1.5, 4.0), (0.0, -1.5, 4.0))),
    "c5s": dict(desc="C5 stochastic: synthetic 16x16 UV-sphere grid OBJ (1,015,810 tris) 3840x2160, 4 jittered "
                     "samples/pixel (RT_STOCHASTIC, seed 0x5EED: pf 2 strata, counter-hash jitter; an extension of "
                     "the reference's regular grid), depth 3, 4 lights",
                scene="syn:C5", width=3840, height=2160, pf=2, max_lvl=3, stochastic=True,
                lights=((0.0, 0.0, 4.0), (1.5, 1.5, 4.0), (-1.5, 1.5, 4.0), (0.0, -1.5, 4.0))),
}


def workload_scene(spec, workdir):
    """Scene file for a workload: synthetic scenes are regenerated; reference models come from the
    gzip'd data fixtures in tests/golden/models (the reference tree is not on the GPU box)."""
    from raytracert_amd import scenes
    kind, name = spec.split(":", 1)
    if kind == "syn":
        if name == "balls":
            return scenes.balls_surrogate(workdir)
        return scenes.write_sphere_grid(getattr(scenes, name), workdir, name.lower())
    sys.path.insert(0, os.path.join(HERE, "tests"))
    from _util import materialize_models
    materialize_models(workdir)
    return os.path.join(workdir, name)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=("weak", "strong"), default="weak")
    ap.add_argument("--cpu-sample-every", type=int, default=96, help="CPU baseline: every k-th tile")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=1, help="steps re-run with HIP events for the roofline")
    ap.add_argument("--ppm", default="", help="write the first frame to this PPM (rank 0)")
    ap.add_argument("--accel", choices=("bvh", "brute_force"), default="bvh")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c4")
    ap.add_argument("--no-bf-roofline", action="store_true", help="skip the brute-force kernel's roofline frame")
    ap.add_argument("--pipes", type=int, default=1, help="render pipelines a call's batches overlap on")
    ap.add_argument("--tune", action="append", default=[], metavar="KNOB=VALUE",
                    help="extra launch-shape knob (Scene.tune), e.g. shadow_virtual=-1; repeatable")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} differs from --gpus {args.gpus}; using WORLD_SIZE")

    import numpy as np
    import torch
    import torch.distributed as dist

    import raytracert_amd as R
    from raytracert_amd import dist as rdist, scenes
    from raytracert_amd._capi import KERNEL_CLOSEST_HIT, KERNEL_SHADOW, KERNEL_SHADE, KERNEL_FRAME, KERNEL_CHAIN

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    wl = WORKLOADS[args.workload]
    WIDTH, HEIGHT, PF, MAX_LVL, LIGHTS = wl["width"], wl["height"], wl["pf"], wl["max_lvl"], wl["lights"]
    tmp = tempfile.mkdtemp(prefix=f"rtbench_r{rank}_")
    t_gen = time.time()
    obj = workload_scene(wl["scene"], tmp)
    t_gen = time.time() - t_gen
    t_load = time.time()
    scene = R.Scene.load(obj, device=local_rank)
    scene.set_accel(args.accel)
    scene.tune("pipes", args.pipes)
    for kv in args.tune:
        k, v = kv.split("=", 1)
        scene.tune(k, int(v, 0))
    t_load = time.time() - t_load
    bvh_info = scene.bvh_info() if args.accel == "bvh" else None
    nv, nt, nm = scene.counts()
    flags = R.ALL_FEATURES | (R._capi.STOCHASTIC if wl.get("stochastic") else 0)
    params = R.RenderParams(width=WIDTH, height=HEIGHT, pf=PF, max_lvl=MAX_LVL, lights=LIGHTS, flags=flags)
    cparams = params.to_c()

    layout = rdist.TileLayout(WIDTH, HEIGHT, TILE, TILE)
    plan = rdist.ShardPlan(layout, world, frames=world if args.mode == "weak" else 1)
    # two shard buffers: step i renders into bufs[i % 2] while step i-1's gather reads the other
    bufs = [torch.zeros(plan.shard_bytes, dtype=torch.uint8, device=dev) for _ in range(2)]
    index = torch.as_tensor(plan.gather_index(), device=dev)
    stream = torch.cuda.current_stream(dev)

    def render_shard(want_counts=False, buf=None):
        # one call: this rank's tile ids rank, rank + N, ... over the step's `frames` frames
        buf = bufs[0] if buf is None else buf
        n, c = scene.render_tiles_device(cparams, TILE, TILE, rank, world, buf.data_ptr(), buf.numel(),
                                         stream.cuda_stream, want_counts=want_counts, frames=plan.frames)
        assert n == plan.rank_tiles(rank)
        return c if c is not None else np.zeros(3, np.uint64)

    pending = []

    def finish(p):
        # order the stream after the gather, then un-permute on rank 0
        if p is None:
            return None
        gathered, work = p
        if work is not None:
            work.wait()
        return rdist.assemble_plan_torch(gathered, plan, index) if rank == 0 else None

    single = world == 1 and plan.frames == 1
    if single:   # one GPU: the library writes the row-major frame itself (no gather, no un-permute)
        fbufs = [torch.zeros(HEIGHT * WIDTH * 3, dtype=torch.uint8, device=dev) for _ in range(2)]

    def step(i):
        """Render step i's shard, start its gather (async, on the collective's stream) and finish
        step i-1's: the gather of one step overlaps the next step's render."""
        if single:
            fb = fbufs[i % 2]
            scene.render_frame_device(cparams, TILE, TILE, fb.data_ptr(), fb.numel(), stream.cuda_stream)
            return fb.view(1, HEIGHT, WIDTH, 3)
        render_shard(buf=bufs[i % 2])
        pending.append(rdist.gather_shards(bufs[i % 2], rank, world, async_op=True))
        return finish(pending.pop(0)) if len(pending) > 1 else None

    def drain():
        return finish(pending.pop(0)) if pending else None

    # rays per step (deterministic): counted once, summed over ranks
    counts = render_shard(want_counts=True)
    ct = torch.tensor([int(c) for c in counts], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ct)
    rays_per_step = float(ct.sum().item())
    rays_by_kind = [int(x) for x in ct.tolist()]

    for i in range(args.warmup):
        step(i)
    drain()
    torch.cuda.synchronize(dev)

    # ---- timed region ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    frames = None
    for i in range(args.steps):
        f = step(i)
        frames = f if f is not None else frames
    f = drain()   # the last step's gather + un-permute stay inside the timed region
    frames = f if f is not None else frames
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    # ---- kernel timing for the roofline (HIP events on the scene's launch stream) ----
    def profile(steps):
        # kernel durations in isolation: one pipeline, so no launch shares the GPU with another
        scene.tune("pipes", 1)
        scene.reset_stats()
        scene.set_profiling(True)
        for _ in range(max(steps, 1)):
            render_shard()
        torch.cuda.synchronize(dev)
        scene.set_profiling(False)
        st = {k: scene.kernel_stats(k) for k in (KERNEL_CLOSEST_HIT, KERNEL_SHADOW, KERNEL_SHADE, KERNEL_FRAME, KERNEL_CHAIN)}
        work = (0.0, 0.0, 0.0, 0.0)
        if scene.accel() == "bvh":   # work counters slow the kernels: count in a separate, untimed pass
            scene.reset_stats()
            scene.set_profiling(True, count_work=True)
            for _ in range(max(steps, 1)):
                render_shard()
            torch.cuda.synchronize(dev)
            scene.set_profiling(False)
            work = scene.work_stats(KERNEL_CLOSEST_HIT) + scene.work_stats(KERNEL_SHADOW)
        scene.tune("pipes", args.pipes)
        return st, work

    stats, (bvh_tests, bvh_visits, sh_bvh_tests, sh_bvh_visits) = profile(args.profile_steps)
    chain_launches, chain_ms, chain_tests = stats[KERNEL_CHAIN]
    ch_launches, ch_ms, ch_tests = stats[KERNEL_CLOSEST_HIT]
    sh_launches, sh_ms, sh_tests = stats[KERNEL_SHADOW]
    _, shade_ms, _ = stats[KERNEL_SHADE]
    _, frame_ms, _ = stats[KERNEL_FRAME]
    bf = None
    if args.accel == "bvh" and not args.no_bf_roofline and rank == 0:
        scene.set_accel("brute_force")
        bst, _ = profile(1)
        scene.set_accel("bvh")
        l, ms, tests = bst[KERNEL_CLOSEST_HIT]
        bf = {"kernel": "k_closest_hit (brute force, --accel brute_force)", "bound": "valu",
              "achieved": round(tests * FLOP_PER_TEST / (ms / 1e3) / 1e12, 3), "peak": FP32_PEAK_TFLOPS,
              "unit": "TFLOP/s", "frac": round(tests * FLOP_PER_TEST / (ms / 1e3) / 1e12 / FP32_PEAK_TFLOPS, 4),
              "launches": l, "avg_launch_ms": round(ms / max(l, 1), 3), "frame_closest_hit_ms": round(ms, 3)}

    result = None
    if rank == 0:
        total_rays = rays_per_step * args.steps
        value = total_rays / elapsed / 1e6
        queries = ch_tests / max(nt, 1)
        if args.accel == "bvh" and chain_launches > 0:
            # The chain kernel (every step of every sample per lane, RT_TUNE_CHAIN_FROM 0): per
            # primary query 32 B in, per closest-hit query a 32-B chain record out, plus one 64-B
            # record per node visit and per triangle test of its closest-hit and shadow queries
            # (device counters). Roof: memory (HBM peak).
            kname = "k_chain"
            ch_launches, ch_ms = chain_launches, chain_ms   # the roofline's kernel from here on
            queries = rays_by_kind[0] / world * args.profile_steps
            tests_all, visits_all = bvh_tests + sh_bvh_tests, bvh_visits + sh_bvh_visits
            flops = tests_all * FLOP_PER_TEST + visits_all * FLOP_PER_NODE
            ch_bytes = (queries * 32.0 + (rays_by_kind[0] + rays_by_kind[1]) / world * args.profile_steps * 32.0 +
                        (visits_all + tests_all) * 64.0)
            bvh_tests, bvh_visits = tests_all, visits_all
            ch_tests = chain_tests
            bound, unit, peak = "hbm", "GB/s", HBM_PEAK_GBS
            achieved = ch_bytes / (ch_ms / 1e3) / 1e9 if ch_ms > 0 else 0.0
            valu = flops / (ch_ms / 1e3) / 1e12 if ch_ms > 0 else 0.0
        elif args.accel == "bvh":
            # BVH traversal is a dependent gather: per query 32 B in + 20 B out, plus one 64-B
            # record per node visit and per triangle test (device counters). Roof: memory (HBM peak).
            kname = "k_bvh_closest_hit"
            flops = bvh_tests * FLOP_PER_TEST + bvh_visits * FLOP_PER_NODE
            ch_bytes = queries * 52.0 + (bvh_visits + bvh_tests) * 64.0
            bound, unit, peak = "hbm", "GB/s", HBM_PEAK_GBS
            achieved = ch_bytes / (ch_ms / 1e3) / 1e9 if ch_ms > 0 else 0.0
            valu = flops / (ch_ms / 1e3) / 1e12 if ch_ms > 0 else 0.0
        else:
            # brute force: each wave streams every 64-B record once (scalar loads); VALU-bound
            kname = "k_closest_hit"
            flops = ch_tests * FLOP_PER_TEST
            ch_bytes = ch_tests / 64.0 * 64.0 + queries * 52.0
            bound, unit, peak = "valu", "TFLOP/s", FP32_PEAK_TFLOPS
            achieved = flops / (ch_ms / 1e3) / 1e12 if ch_ms > 0 else 0.0
            valu = achieved
        # the committed PMC summary profiles the default workload (C4): other workloads carry none
        traffic, traffic_src = pmc_traffic(kname) if args.workload == "c4" else (None, None)
        result = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "weak" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": wl["desc"],
                "frames_per_step": plan.frames,
                "width": WIDTH, "height": HEIGHT, "pf": PF, "max_lvl": MAX_LVL, "lights": [list(l) for l in LIGHTS],
                "triangles": nt, "vertices": nv, "tile": TILE,
                "parallelism": f"tile-shard{world}",
                "rays_per_step": int(rays_per_step),
                "rays_by_kind_per_step": {"primary": rays_by_kind[0], "secondary": rays_by_kind[1], "shadow": rays_by_kind[2]},
                "frame_ms_per_gpu": round(elapsed / args.steps * 1e3, 3),
                "scene_load_s": round(t_load, 3), "scene_gen_s": round(t_gen, 3),
            },
            "roofline": {
                "kernel": f"{kname} ({'every chain step: closest-hit, shadow and shade' if kname == 'k_chain' else 'primary + secondary queries'}, accel={args.accel})",
                "bound": bound,
                "achieved": round(achieved, 3),
                "peak": peak,
                "unit": unit,
                "frac": round(achieved / peak, 4),
                "algorithmic_bytes_per_launch": round(ch_bytes / max(ch_launches, 1)),
                "valu_TFLOPs": round(valu, 3),
                "valu_frac": round(valu / FP32_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "traffic_unit": "bytes/launch (PMC: 2*FETCH_SIZE + WRITE_SIZE)",
                "traffic_source": traffic_src,
                "launches": ch_launches,
                "avg_launch_ms": round(ch_ms / max(ch_launches, 1), 3),
                "queries_per_launch": round(queries / max(ch_launches, 1)),
                "tests_per_launch": round((bvh_tests if args.accel == "bvh" else ch_tests) / max(ch_launches, 1)),
                "node_visits_per_launch": round(bvh_visits / max(ch_launches, 1)) if args.accel == "bvh" else 0,
                "flop_per_test": FLOP_PER_TEST,
                "flop_per_node_visit": FLOP_PER_NODE,
                "bruteforce_equivalent_TFLOPs": round(ch_tests * FLOP_PER_TEST / (ch_ms / 1e3) / 1e12, 3) if ch_ms > 0 else None,
            },
            "kernel_ms_per_step": {
                "closest_hit": round(stats[KERNEL_CLOSEST_HIT][1] / max(args.profile_steps, 1), 3),
                "shadow": round(sh_ms / max(args.profile_steps, 1), 3),
                "shade": round(shade_ms / max(args.profile_steps, 1), 3),
                "frame": round(frame_ms / max(args.profile_steps, 1), 3),
                "chain": round(chain_ms / max(args.profile_steps, 1), 3),
            },
            "roofline_bruteforce": bf,
            "accel": {"mode": args.accel, "bvh": bvh_info},
            "cpu_baseline": None,
        }
        if args.ppm and frames is not None:
            R.write_ppm(args.ppm, frames[0].cpu().numpy())

    # ---- CPU baseline + in-run parity on a bounded tile sample (rank 0, N=1 only) ----
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(obj, params, frames[0].cpu().numpy(), layout, args, wl)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/*_pmc.json,
    written by tools/pmc_summary.py from separate rocprofv3 --pmc passes of this bench command)."""
    import glob
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "*_pmc.json")))   # round-tagged names sort by age
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        ks = d.get("kernels", {})
        # the timed (non-counting) instantiation of the kernel, e.g. "k_bvh_closest_hit<4, false>"
        names = [n for n in ks if n == kernel or (n.startswith(kernel + "<") and n.endswith("false>"))]
        for n in names:
            if "traffic_bytes_per_launch" in ks[n]:
                return ks[n]["traffic_bytes_per_launch"], os.path.relpath(f, HERE)
    return None, None


def cpu_baseline(obj, params, gpu_frame, layout, args, wl):
    """Time the CPU restatement (oracle/, 'port') on every k-th 16x16 tile of the same frame with
    --cpu-threads threads, and check the GPU's bytes on those tiles against it."""
    import numpy as np
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle as O
    sc = O.OracleScene(obj)
    op = O.make_params(params.width, params.height, params.pf, params.max_lvl, lights=params.lights, flags=params.flags,
                       seed=params.seed)
    tiles = list(range(0, layout.n_tiles, args.cpu_sample_every))
    threads = args.cpu_threads
    rays = 0
    max_d = 0
    exact = 0
    total = 0
    t0 = time.perf_counter()
    outs = []
    for t in tiles:
        ty, tx = divmod(t, layout.tiles_x)
        x0, y0 = tx * layout.tile_w, ty * layout.tile_h
        w = min(layout.tile_w, params.width - x0)
        h = min(layout.tile_h, params.height - y0)
        _, u8, c = sc.render(op, x0, y0, w, h, nthreads=threads)
        rays += int(c.sum())
        outs.append((x0, y0, w, h, u8))
    dt = time.perf_counter() - t0
    for x0, y0, w, h, u8 in outs:
        g = gpu_frame[y0:y0 + h, x0:x0 + w]
        d = np.abs(g.astype(np.int16) - u8.astype(np.int16))
        max_d = max(max_d, int(d.max()))
        exact += int((d == 0).sum())
        total += d.size
    import platform
    return {
        "value": round(rays / dt / 1e6, 6),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{len(tiles)} of {layout.n_tiles} 16x16 tiles (every {args.cpu_sample_every}th) of the same "
                  f"{wl['desc'].split(':')[0]} frame, {rays} rays in {dt:.1f} s, oracle/rt_oracle.c (-O2) on {threads} threads, "
                  f"host {platform.processor() or platform.machine()}",
        "parity_vs_gpu": {"bytes": total, "exact_frac": round(exact / max(total, 1), 6), "max_lsb": max_d},
    }


if __name__ == "__main__":
    main()
