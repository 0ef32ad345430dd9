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
TEST_STAGE_FLOPS = (14, 1, 23, 5, 9)   # per stage a test reaches (rt_kernels.hip kTestStageFlops; brute-force roofline)
FLOP_PER_NODE = 52            # BVH node visit: 2 slab tests (6 sub + 6 mul + 12 min/max each) + 2 distance culls
FP32_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 vector (= FP32 matrix) peak (packed FMA)
# The same issue rate without packing (x2) or FMA (x2), which parity forbids for the triangle test:
# 256 CUs x 64 lanes x 2.4 GHz x 1 flop = 39.3 TFLOP/s (the brute-force kernel's practical ceiling)
FP32_NOFMA_NOPACK_TFLOPS = 39.3
VALU_CYCLES_PER_WAVE_INST = 4   # wave64 non-packed FP32 op on one SIMD (tools/valu_rate.hip: 38.7 T lane-ops/s)
CLOCK_HZ = 2.4e9
HBM_PEAK_GBS = 8000.0
TILE = 16
LEG_STEPS = 100   # frames the modes beside the headline time at least (one at a time, two in flight, the orbit)
# BASELINE.json configs. C4 is the metric's configuration and the default; the
# others are available with --workload (C1 is the reference's own CPU-only plumbing case).
WORKLOADS = {
    "c4": dict(desc="C4: synthetic 8x8 UV-sphere grid OBJ (102,402 tris) 1920x1080, pf 1, depth 3, 2 lights",
               scene="syn:C4", width=1920, height=1080, pf=1, max_lvl=3, lights=((0.0, 0.0, 4.0), (1.5, 1.5, 4.0)),
               cpu_every=96, dropin=True, dropin_keys=("-", "-", "M:3", "A:1.5,1.5,4")),
    "c2": dict(desc="C2: dodgeColorTest.obj (16,311 tris) 800x600, pf 1, depth 1, 1 light",
               scene="ref:dodgeColorTest.obj", width=800, height=600, pf=1, max_lvl=1, lights=((0.0, 0.0, 4.0),),
               cpu_every=1),
    "c3": dict(desc="C3: Balls surrogate (3 UV spheres 48x24 + ground quad, Balls.mtl materials) 1920x1080, pf 1, "
                    "depth 3, 2 lights (Balls.obj is missing from the reference)",
               scene="syn:balls", width=1920, height=1080, pf=1, max_lvl=3, lights=((0.0, 0.0, 4.0), (2.0, 2.0, 4.0)),
               cpu_every=16),
    "c5": dict(desc="C5: synthetic 16x16 UV-sphere grid OBJ (1,015,810 tris) 3840x2160, pf 2 (4 samples/pixel, "
                    "the reference's regular AA grid), depth 3, 4 lights",
               scene="syn:C5", width=3840, height=2160, pf=2, max_lvl=3,
               lights=((0.0, 0.0, 4.0), (1.5, 1.5, 4.0), (-1.5, 1.5, 4.0), (0.0, -1.5, 4.0)), cpu_every=1024),
    "ref_default": dict(desc="the reference's own defaults: dodgeColorTest.obj (16,311 tris) 500x500 window, pixelfactor 3 "
                             "(9 sub-samples/pixel), max_lvl 10, light 0 = the camera (main.cpp:137-141, "
                             "raytracing.cpp:23-29,72)",
                        scene="ref:dodgeColorTest.obj", width=500, height=500, pf=3, max_lvl=10, lights=((0.0, 0.0, 4.0),),
                        cpu_every=4, dropin=True),
    "c5s": dict(desc="C5 stochastic: synthetic 16x16 UV-sphere grid OBJ (1,015,810 tris) 3840x2160, 4 jittered "
                     "samples/pixel (RT_STOCHASTIC, seed 0x5EED: pf 2 strata, counter-hash jitter; an extension of "
                     "the reference's regular grid), depth 3, 4 lights",
                scene="syn:C5", width=3840, height=2160, pf=2, max_lvl=3, stochastic=True,
                lights=((0.0, 0.0, 4.0), (1.5, 1.5, 4.0), (-1.5, 1.5, 4.0), (0.0, -1.5, 4.0)), cpu_every=1024),
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
    ap.add_argument("--e2e-inflight", type=int, default=2)   # renders in flight in the full line's end-to-end leg (r06as: 0.37-0.48 vs 0.50-0.66 ms with one)
    ap.add_argument("--steps", type=int, default=100)   # ~50 ms of C4 frames: fixed sync costs amortised
    ap.add_argument("--warmup", type=int, default=20)   # (the launch trials run before it: calibration)
    ap.add_argument("--mode", choices=("weak", "strong"), default="weak")
    ap.add_argument("--cpu-sample-every", type=int, default=0,
                    help="CPU baseline: every k-th tile (0: the workload's default, C2 the full frame)")
    ap.add_argument("--cpu-threads", type=int, default=16, help="the GPU box's CPU share (16 per GPU)")
    ap.add_argument("--cpu-single-budget", type=float, default=15.0,
                    help="1-thread CPU figure: seconds spent on 4x4-pixel blocks of the sampled tiles")
    ap.add_argument("--comm", choices=("torch", "rt"), default="torch",
                    help="N>1 gather: torch.distributed (RCCL) + the library's un-permute kernel, or the library's own "
                         "RCCL communicator end to end (rt_render_frames_sharded)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 rehearsal on ONE GPU: every rank renders on device 0 and the collectives run over "
                         "gloo with host staging (checks the multi-rank logic where RCCL refuses two ranks per GPU; "
                         "timings are not scaling numbers)")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold (unordered) first-frame measurement")
    ap.add_argument("--no-path-compare", action="store_true",
                    help="N=1: skip timing the shard path (tiles + un-permute) beside the frame path")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="ref_default: skip timing the drop-in's literal 'r' loop")
    ap.add_argument("--profile-steps", type=int, default=20, help="frames re-run with HIP events for the roofline (averaged)")
    ap.add_argument("--ppm", default="", help="write the first frame to this PPM (rank 0)")
    ap.add_argument("--accel", choices=("bvh", "brute_force"), default="bvh")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c4")
    ap.add_argument("--no-bf-roofline", action="store_true", help="skip the brute-force kernel's roofline frame")
    ap.add_argument("--pipes", type=int, default=1, help="render pipelines a call's batches overlap on")
    ap.add_argument("--inflight", type=int, default=1,
                    help="N=1 frame path: calls in flight (RT_TUNE_FRAMES_IN_FLIGHT), consecutive calls on this many "
                         "alternating streams into their own buffers (r06: 1; with the camera path's distinct views, two "
                         "four-view calls in flight measured 0.339-0.347 ms per frame against 0.331-0.332 one call at a "
                         "time, profiles/r06e_ab_headline.txt)")
    ap.add_argument("--orbit-step", type=float, default=0.25,
                    help="N=1: also time a moving view, each frame the view turned by this many degrees more "
                         "(scenes.orbit_corners; 0 = skip): config.orbit")
    ap.add_argument("--no-multi-frame", action="store_true", help="skip the rt_render_frames_device leg")
    ap.add_argument("--frames-per-call", type=int, default=8,
                    help="N=1 frame path: frames per rt_render_frames_device call (one chain launch), 1-8 (r06: 8, "
                         "0.320-0.322 ms per frame against 0.325-0.327 at 4, profiles/r06i_ab_views_per_call.txt)")
    ap.add_argument("--camera-path", type=float, default=0.25,
                    help="N=1 with --frames-per-call > 1: the frames of a call are consecutive views of a camera path "
                         "around the default view (turned -4..4 x this many degrees about y, a triangle wave of period "
                         "16), so no two frames of a call are the same view (ADVICE r05); 0 = the same view K times")
    ap.add_argument("--no-strong-shares", action="store_true",
                    help="N=1: skip timing rank r's 1/N share of one frame for N = 2, 4, 8 (strong_shares)")
    ap.add_argument("--no-e2e", action="store_true", help="N=1: skip the end-to-end frame (render -> host -> PPM file)")
    ap.add_argument("--e2e-only", action="store_true", help="N=1: only the end-to-end frame leg (one JSON line)")
    ap.add_argument("--e2e-frames", type=int, default=40, help="frames of the end-to-end leg per mode")
    ap.add_argument("--ppm-threads", type=int, default=8, help="end-to-end leg: threads writing each PPM (rt_ppm_writer)")
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

    if args.rehearse:   # every rank on device 0, gloo collectives on host copies
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        if args.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def all_reduce(t, op=None):
        """dist.all_reduce on a device tensor (host-staged over gloo when rehearsing)."""
        op = dist.ReduceOp.SUM if op is None else op
        if not args.rehearse:
            dist.all_reduce(t, op=op)
            return
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)

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
    stream = torch.cuda.current_stream(dev)
    rtcomm = None
    if args.comm == "rt":   # the library's communicator: rank 0's id broadcast over torch.distributed
        uid = torch.zeros(R._capi.COMM_ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(R.Comm.unique_id()), dtype=torch.uint8))
        if world > 1:
            if args.rehearse:
                raise SystemExit("--comm rt needs one GPU per rank (RCCL refuses two ranks on one device)")
            dist.broadcast(uid, 0)
        rtcomm = R.Comm(local_rank, rank, world, bytes(uid.cpu().numpy().tobytes()))

    class Runner:
        """One way of rendering a step. frames: frames per step (weak: N, strong: 1); frame_path:
        one GPU writes the row-major frame itself (rt_render_frame_device: no gather, no
        un-permute); otherwise every rank renders its interleaved tiles (rt_render_tiles_device),
        rank 0 gathers them (one RCCL gather) and un-permutes them on the device."""

        def __init__(self, frames, frame_path):
            self.plan = rdist.ShardPlan(layout, world, frames=frames)
            self.single = frame_path
            # two buffers: step i renders into bufs[i % 2] while step i-1's gather reads the other
            self.bufs = [torch.zeros(self.plan.shard_bytes, dtype=torch.uint8, device=dev) for _ in range(2)]
            self.index = torch.as_tensor(self.plan.gather_index(), device=dev)
            if frame_path:
                self.fbufs = [torch.zeros(HEIGHT * WIDTH * 3, dtype=torch.uint8, device=dev)
                              for _ in range(max(2, args.inflight, 2 * args.frames_per_call))]
                # frames in flight: frame i on stream i % F (the first is the bench's stream). (Streams on
                # hardware queues of their own, CU-masked, made the frames overlap worse: 0.43-0.52 vs
                # 0.35 ms per C4 frame, profiles/r05e_ab_rtstreams.txt)
                self.fstreams = [stream] + [torch.cuda.Stream(dev) for _ in range(max(args.inflight, 2) - 1)]   # (>= 2: the in-flight leg)
                # a new stream's first command initialises it (~6 ms of host time on this image): done
                # here, at setup, not at the warm-up's second frame, where it left the GPU idle just
                # before the timed frames (they then ran ~5% slow for ~25 frames)
                for fs in self.fstreams[1:]:
                    with torch.cuda.stream(fs):
                        torch.zeros(1, device=dev).add_(1)
                torch.cuda.synchronize(dev)
            elif rank == 0:
                self.frames_out = [torch.zeros(frames * HEIGHT * WIDTH * 3, dtype=torch.uint8, device=dev) for _ in range(2)]
            else:
                self.frames_out = [torch.zeros(1, dtype=torch.uint8, device=dev)] * 2
            self.kstep = 1   # N > 1 weak: steps per render call (the plan holds kstep x N frames)
            self.fif = 1   # frames in flight of the current run (the timed run sets args.inflight)
            self.fpc = 1   # frames per call (rt_render_frames_device; the timed run sets --frames-per-call)
            self.total = 0   # frames of the current run's timed steps (frame path: steps are calls of fpc frames)
            self.nfin = 0
            self.pending = []
            self.path = None       # camera path views (c params) of the multi-frame headline, and their ray counts
            self.path_rays = None
            self.pidx = 0          # next path position
            self.rays_acc = 0      # rays of the path views rendered since the last reset
            self.last_pos = 0      # path position of the last rendered frame
            # rank 0 un-permutes on a side stream, so the next step's render is not queued behind it
            self.side = torch.cuda.Stream(dev) if (rank == 0 and not frame_path) else None

        def render_shard(self, want_counts=False, buf=None):
            # one call: this rank's tile ids rank, rank + N, ... over the step's `frames` frames
            buf = self.bufs[0] if buf is None else buf
            n, c = scene.render_tiles_device(cparams, TILE, TILE, rank, world, buf.data_ptr(), buf.numel(),
                                             stream.cuda_stream, want_counts=want_counts, frames=self.plan.frames)
            assert n == self.plan.rank_tiles(rank)
            return c if c is not None else np.zeros(3, np.uint64)

        def render_once(self, i=0):
            """The step's render call alone (the roofline's profiled launches use this)."""
            if self.single:
                fb = self.fbufs[i % max(2, self.fif)]
                st = self.fstreams[i % self.fif]
                scene.render_frame_device(cparams, TILE, TILE, fb.data_ptr(), fb.numel(), st.cuda_stream)
                return fb
            return self.render_shard(buf=self.bufs[i % 2])

        def finish(self, p):
            # order the render stream after the gather (the next render reuses the gathered shard
            # buffer; the gather is long done by then), then un-permute on rank 0's side stream
            # (the library's kernel), which waits for the same point
            gathered, work = p
            if work is not None:
                work.wait()
            if rank != 0:
                return None
            out = self.frames_out[self.nfin % 2]
            self.nfin += 1
            ev = torch.cuda.Event()
            ev.record(stream)
            self.side.wait_event(ev)
            gathered.record_stream(self.side)
            R.assemble_tiles_device(local_rank, WIDTH, HEIGHT, TILE, TILE, self.plan.frames, world, gathered.data_ptr(),
                                    gathered.numel(), out.data_ptr(), out.numel(), self.side.cuda_stream)
            return out.view(self.plan.frames, HEIGHT, WIDTH, 3)

        def render_call(self, i, k):
            """Call i of a multi-frame run: k frames of the view in one rt_render_frames_device call
            (one chain launch) into buffers (i % 2) * fpc ..., on stream i % F."""
            base = (i % 2) * self.fpc
            st = self.fstreams[i % self.fif]
            bufs = self.fbufs[base:base + k]
            if self.path is None:
                views = [cparams] * k
            else:   # k consecutive views of the camera path
                pos = [(self.pidx + j) % len(self.path) for j in range(k)]
                views = [self.path[m] for m in pos]
                self.rays_acc += sum(self.path_rays[m] for m in pos)
                self.pidx += k
                self.last_pos = pos[-1]
            scene.render_frames_device(views, TILE, TILE, [b.data_ptr() for b in bufs], bufs[0].numel(), st.cuda_stream)
            return bufs[-1]

        def step(self, i, k=1):
            """Render step i, start its gather (async, on the collective's stream) and finish step
            i-1's: the gather of one step overlaps the next step's render. Frame path with fpc > 1:
            step i is a call of k frames."""
            if self.single:
                if self.fpc > 1:
                    return self.render_call(i, k).view(1, HEIGHT, WIDTH, 3)
                return self.render_once(i).view(1, HEIGHT, WIDTH, 3)
            if rtcomm is not None:   # render + RCCL gather + un-permute, all inside the library
                out = self.frames_out[i % 2]
                scene.render_frames_sharded(cparams, rtcomm, TILE, TILE, self.plan.frames, out.data_ptr() if rank == 0 else None,
                                            out.numel() if rank == 0 else 0, stream.cuda_stream)
                return out.view(self.plan.frames, HEIGHT, WIDTH, 3) if rank == 0 else None
            self.render_shard(buf=self.bufs[i % 2])
            if args.rehearse and world > 1:   # host-staged gather over gloo (synchronous)
                torch.cuda.synchronize(dev)
                h = self.bufs[i % 2].cpu()
                parts = [torch.empty_like(h) for _ in range(world)] if rank == 0 else None
                dist.gather(h, parts, dst=0)
                self.pending.append((torch.cat(parts).to(dev) if rank == 0 else None, None))
            else:
                self.pending.append(rdist.gather_shards(self.bufs[i % 2], rank, world, async_op=True))
            return self.finish(self.pending.pop(0)) if len(self.pending) > 1 else None

        def drain(self):
            return self.finish(self.pending.pop(0)) if self.pending else None

        def run(self, steps, warmup):
            """warmup untimed steps, then `steps` timed ones between barriers + device syncs;
            returns (max-over-ranks seconds, last frames). Frame path with fpc > 1: `steps` frames
            as calls of fpc frames (the last call the remainder); self.total = frames timed."""
            calls = [self.fpc] * (steps // self.fpc) + ([steps % self.fpc] if steps % self.fpc else []) \
                if (self.single and self.fpc > 1) else [1] * (steps // self.kstep)
            self.total = sum(calls)
            for i in range(warmup if self.single else max(1, warmup // self.kstep) if warmup else 0):
                self.step(i, self.fpc)
            self.drain()
            self.rays_acc = 0
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            frames = None
            for i, k in enumerate(calls):
                f = self.step(i, k)
                frames = f if f is not None else frames
            f = self.drain()   # the last step's gather + un-permute stay inside the timed region
            frames = f if f is not None else frames
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            if world > 1:
                all_reduce(el, dist.ReduceOp.MAX)
            return float(el.item()), frames

    # N > 1, weak scaling: a render call covers --frames-per-call steps (each rank's share of that many
    # steps' N frames in one launch, one gather, one un-permute), as the one-GPU line renders that many
    # frames per call; the step count must be a whole number of calls, else one step per call
    kstep = 1
    if world > 1 and args.mode == "weak" and rtcomm is None and args.frames_per_call > 1:
        # the largest step count per call up to --frames-per-call that divides the timed steps
        kstep = max(d for d in range(1, min(args.frames_per_call, 8) + 1) if args.steps % d == 0)
    main_run = Runner(world * kstep if args.mode == "weak" else 1, frame_path=world == 1 and rtcomm is None)
    main_run.kstep = kstep
    plan = main_run.plan

    # rays per step (deterministic): counted once, summed over ranks
    counts = main_run.render_shard(want_counts=True)
    ct = torch.tensor([int(c) for c in counts], dtype=torch.float64, device=dev)
    if world > 1:
        all_reduce(ct)
    rays_per_step = float(ct.sum().item()) / kstep
    rays_by_kind = [int(x) // kstep for x in ct.tolist()]

    # ---- calibration: the view's per-view launch trials (rt_scene_trials) run on pipeline 0, one
    # frame at a time, before any timed or warm-up frame: a new view's first ~20 launches include
    # the batch-order settling and the trial launches (some of them slow candidates by design), which
    # a renderer serving a view pays once. Bounded; the count is reported (config.calibration_frames).
    inflight = max(1, args.inflight) if main_run.single else 1

    def calibrate(fif):
        # frames one at a time (synchronised: a trial is decided once its launches' events have
        # completed), alternating over the F pipelines of the timed mode: pipeline 0's launches run the
        # trials, the others adopt its order and decision, and every pipeline's one-time setup
        # (workspace, streams) happens here rather than just before the timed frames (an idle GPU there
        # left the next ~25 frames ~5% slow: the clock ramps back up, profiles/r04_inflight_settle.txt)
        n = 0
        if args.accel == "bvh" and rtcomm is None:   # (each rank its own view's trials, before the barrier)
            while n < 64 * fif and scene.trials()["choice"] < 0:
                main_run.render_once(n)
                n += 1
                torch.cuda.synchronize(dev)
            for _ in range((fif - n % fif) % fif):   # (end on a whole round: timed frame i takes pipeline i mod F)
                main_run.render_once(n)
                n += 1
                torch.cuda.synchronize(dev)
        return n

    if inflight > 1:
        # the other pipelines start from pipeline 0's batch order and adopt its trial decision
        # (rt_capi.cpp run_chain); call i after the tune takes pipeline i mod F
        scene.tune("frames_in_flight", inflight)
        main_run.fif = inflight
    calib = calibrate(inflight)
    if args.e2e_only:   # the end-to-end leg alone (tools/gpu_run.sh e2e)
        scene.tune("frames_in_flight", 1)
        calibrate(1)
        e2e = {f"renders_in_flight_{k}": end_to_end(scene, cparams, WIDTH, HEIGHT, dev, frames=args.e2e_frames,
                                                      threads=args.ppm_threads, workdir=tmp, inflight=k) for k in (1, 2)}
        if rank == 0:
            print(json.dumps({"metric": "end-to-end wall clock per frame", "workload": wl["desc"], "end_to_end": e2e}), flush=True)
        return
    fpc = max(1, min(args.frames_per_call, 8)) if main_run.single else 1
    main_run.fpc = fpc
    path_what = None
    if fpc > 1 and args.camera_path > 0:
        # the headline's camera path: view m of 16 = the default view turned by tri(m) x step degrees about
        # the world y axis (the trackball's effect on produceRay, scenes.orbit_corners), tri = 0,1,..,4,3,..,-4,..,-1
        tri = [m if m <= 4 else 8 - m if m <= 12 else m - 16 for m in range(16)]
        main_run.path = [R.RenderParams(width=WIDTH, height=HEIGHT, pf=PF, max_lvl=MAX_LVL, lights=LIGHTS, flags=flags,
                                        corners=scenes.orbit_corners(WIDTH, HEIGHT, t, args.camera_path)).to_c() for t in tri]
        per_angle = {}
        fbc = main_run.fbufs[0]
        for t in sorted(set(tri)):
            c = scene.render_frame_device(main_run.path[tri.index(t)], TILE, TILE, fbc.data_ptr(), fbc.numel(),
                                          stream.cuda_stream, want_counts=True)
            per_angle[t] = int(sum(int(x) for x in c))
        main_run.path_rays = [per_angle[t] for t in tri]
        path_what = {"views": 16, "distinct": len(per_angle), "step_deg": args.camera_path,
                     "turn_deg": [round(t * args.camera_path, 4) for t in tri],
                     "rays_per_view": {str(round(t * args.camera_path, 4)): r for t, r in per_angle.items()},
                     "what": "the timed calls render consecutive views of this camera path around the default view "
                             "(four distinct views per call); rays are counted per view"}
    # ---- timed region (the metric) ----
    elapsed, frames = main_run.run(args.steps, args.warmup * inflight)
    main_run.fpc = 1
    # the last timed frame, kept before any later leg reuses its buffer: the in-run parity check
    # (cpu_baseline) reads this copy, at that frame's view (a camera-path view in the headline mode)
    timed_last = frames.clone() if frames is not None else None
    timed_corners = timed_corners_deg = None
    timed_rays = main_run.rays_acc if main_run.path is not None else None
    if main_run.path is not None:
        tri_last = [m if m <= 4 else 8 - m if m <= 12 else m - 16 for m in range(16)][main_run.last_pos]
        timed_corners = scenes.orbit_corners(WIDTH, HEIGHT, tri_last, args.camera_path)
        timed_corners_deg = round(tri_last * args.camera_path, 4)
    headline_path = main_run.path
    main_run.path = None   # (the other legs render the default view; the roofline's profiled calls the path again)
    torch.cuda.synchronize(dev)
    timed_last_what = (f"the last frame of the last timed call ({fpc} frames per call, {inflight} call(s) in flight"
                       + (f", camera-path view turned {timed_corners_deg} degrees)" if timed_corners is not None else ")")
                       if main_run.single else f"timed step {args.steps - 1} of {args.steps} (the assembled frame on rank 0)")
    one_in_flight = in_flight = None
    value_mode = (f"{fpc}_frames_per_call" if fpc > 1 else "") + (f"{'_' if fpc > 1 else ''}{inflight}_in_flight" if inflight > 1 else "")
    value_mode = (value_mode or "one_in_flight") + ("_camera_path" if timed_rays else "")
    # (the modes beside the headline time at least LEG_STEPS frames, whatever --steps the headline takes: a run of
    # 20 frames one at a time reads ~6% above the steady state, its first launch and last sync unamortised)
    leg_steps, leg_warm = max(args.steps, LEG_STEPS), max(args.warmup, 20)
    if main_run.single and (inflight > 1 or fpc > 1):   # the same frames one at a time (each frame's own latency)
        scene.tune("frames_in_flight", 1)
        main_run.fif = 1
        el1, _ = main_run.run(leg_steps, leg_warm)
        one_in_flight = {"ms_per_step": round(el1 / leg_steps * 1e3, 3),
                         "value": round(rays_per_step * leg_steps / el1 / 1e6, 4), "frames": leg_steps,
                         "what": "the same timed loop with one frame per call and one in flight (each launch waits for "
                                 "the previous frame)"}
        if fpc > 1:   # and one frame per call, two calls in flight on two streams (round 4's headline mode)
            scene.tune("frames_in_flight", 2)
            main_run.fif = 2
            el2, _ = main_run.run(leg_steps, leg_warm * 2)
            in_flight = {"ms_per_step": round(el2 / leg_steps * 1e3, 3), "value": round(rays_per_step * leg_steps / el2 / 1e6, 4),
                         "frames": leg_steps,
                         "what": "one frame per call, two frames in flight on alternating streams (RT_TUNE_FRAMES_IN_FLIGHT 2)"}
            scene.tune("frames_in_flight", 1)
            main_run.fif = 1
        # the line's value is the configured mode's (--frames-per-call, --inflight: chosen before the run);
        # the other modes over the same frames are reported beside it

    # ---- several frames per call (rt_render_frames_device): one launch, one stream ----
    multi_frame = None
    if main_run.single and args.accel == "bvh" and not args.no_multi_frame:
        multi_frame = multiframe_leg(scene, main_run, cparams, WIDTH, HEIGHT, args, rays_per_step, dev)

    # ---- a moving view: every frame a new view of an orbit (the trackball turned, then 'r') ----
    orbit = None
    if main_run.single and args.orbit_step > 0 and args.accel == "bvh":
        orbit = orbit_leg(scene, main_run, WIDTH, HEIGHT, PF, MAX_LVL, LIGHTS, flags, args, inflight, obj, dev)
    orbit_last = orbit.pop("_last") if orbit else None

    rehearsal = None
    if args.rehearse and rank == 0 and frames is not None:   # every assembled frame = the one-GPU frame
        fb = torch.zeros(HEIGHT * WIDTH * 3, dtype=torch.uint8, device=dev)
        scene.render_frame_device(cparams, TILE, TILE, fb.data_ptr(), fb.numel(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ref = fb.view(HEIGHT, WIDTH, 3)
        rehearsal = {"frames_checked": int(frames.shape[0]),
                     "all_equal_one_gpu_frame": bool(all(torch.equal(frames[f], ref) for f in range(frames.shape[0]))),
                     "note": "ranks share one GPU; gloo host-staged gather: logic check, not a scaling number"}

    # ---- a cold frame: the first frame of a new view (no measured batch order, no launch trial):
    # the library dispatches it centre-out (RT_TUNE_COLD_ESTIMATE 2); for comparison the same frame
    # dispatched in screen order ----
    def cold_frame(i):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        scene.tune("forget_order", 1)
        t0 = time.perf_counter()
        main_run.step(i)
        main_run.drain()
        if main_run.single:
            # the frame is done when its stream is: the library's re-sort of the launch's durations (for
            # the next frame) runs on a side stream of its own, which a device-wide sync would also wait for
            for fs in main_run.fstreams:
                fs.synchronize()
            el = time.perf_counter() - t0
            torch.cuda.synchronize(dev)
            return el
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    trials = scene.trials() if hasattr(R._capi.lib(), "rt_scene_trials") else None   # the timed loop's launch shape
    cold = [cold_frame(i) for i in range(0 if args.no_cold else 3)]
    scene.tune("cold_estimate", 0)
    cold_screen = [cold_frame(i) for i in range(0 if args.no_cold else 3)]
    scene.tune("cold_estimate", 2)   # (the library default)
    cold_ms = sorted(cold)[1] * 1e3 if cold else None
    cold_screen_ms = sorted(cold_screen)[1] * 1e3 if cold_screen else None
    # ---- strong scaling measured on this GPU: rank r's 1/N share of one frame, every r, N = 2, 4, 8 ----
    shares = None
    if world == 1 and args.accel == "bvh" and not args.no_strong_shares and not args.rehearse:
        shares = strong_shares(scene, cparams, WIDTH, HEIGHT, dev)
    main_run.run(0, max(args.warmup, 3))   # re-learn the measured order before the other legs
    calibrate(1)                            # (and re-decide the launch trials the cold legs forgot)
    # ---- end to end: render -> bytes in host memory -> result.ppm (main.cpp:347-405) ----
    e2e = None
    if world == 1 and not args.no_e2e and not args.rehearse:
        e2e = end_to_end(scene, cparams, WIDTH, HEIGHT, dev, frames=args.e2e_frames, threads=args.ppm_threads, workdir=tmp,
                         inflight=args.e2e_inflight)
        main_run.run(0, max(args.warmup, 3))

    # ---- the same work through the other path: N=1 the shard path (tiles + un-permute, what
    # N>1 runs, minus the collective); N>1 strong scaling (one frame split over the ranks) ----
    extra = {}
    if world == 1 and not args.no_path_compare and args.accel == "bvh":
        el2, _ = Runner(1, frame_path=False).run(args.steps, max(args.warmup, 2))
        extra["shard_path"] = {"what": "rt_render_tiles_device (interleaved 16x16 tiles) + device un-permute, "
                                       "the N>1 step without its gather", "ms_per_step": round(el2 / args.steps * 1e3, 3),
                               "value": round(rays_per_step * args.steps / el2 / 1e6, 4)}
    if world > 1 and args.mode == "weak":
        srun = Runner(1, frame_path=False)
        el2, _ = srun.run(args.steps, max(args.warmup, 2))
        extra["strong"] = {"what": "one frame split over the N ranks per step (strong scaling)",
                           "ms_per_frame": round(el2 / args.steps * 1e3, 3),
                           "value": round(rays_per_step / world * args.steps / el2 / 1e6, 4)}

    # ---- kernel timing for the roofline (HIP events on the scene's launch stream) ----
    def profile(steps, runner, k=1):
        # kernel durations in isolation: one pipeline, so no launch shares the GPU with another;
        # the same entry point as the timed loop (k frames per call), after it (so every launch is
        # batch-ordered)
        def one(i):
            if k > 1 and runner.single:
                runner.fpc = k
                runner.path = headline_path
                runner.render_call(i, k)
                runner.fpc = 1
                runner.path = None
            else:
                runner.render_once(i)
        scene.tune("pipes", 1)
        one(0)
        torch.cuda.synchronize(dev)
        scene.reset_stats()
        scene.set_profiling(True)
        for i in range(max(steps, 1)):
            one(i)
        torch.cuda.synchronize(dev)
        scene.set_profiling(False)
        st = {k_: scene.kernel_stats(k_) for k_ in (KERNEL_CLOSEST_HIT, KERNEL_SHADOW, KERNEL_SHADE, KERNEL_FRAME, KERNEL_CHAIN)}
        work = (0.0, 0.0, 0.0, 0.0)
        if scene.accel() == "bvh":   # work counters slow the kernels: count in a separate, untimed pass
            scene.reset_stats()
            scene.set_profiling(True, count_work=True)
            for i in range(max(steps, 1)):
                one(i)
            torch.cuda.synchronize(dev)
            scene.set_profiling(False)
            work = scene.work_stats(KERNEL_CLOSEST_HIT) + scene.work_stats(KERNEL_SHADOW)
        scene.tune("pipes", args.pipes)
        return st, work

    stats, (bvh_tests, bvh_visits, sh_bvh_tests, sh_bvh_visits) = profile(args.profile_steps, main_run, fpc)
    # the wave batches of the latest (ordered) launch: the longest is the frame's critical path, the
    # floor of any split of one frame over N GPUs (DESIGN.md §9's strong-scaling model)
    batches = None
    if world == 1 and args.accel == "bvh" and hasattr(R._capi.lib(), "rt_batch_durations"):   # (A/B builds may predate it)
        main_run.render_once()
        bd = scene.batch_durations()
        if bd.size:
            batches = {"n": int(bd.size), "max_us": round(float(bd.max()), 1), "p99_us": round(float(np.percentile(bd, 99)), 1),
                       "median_us": round(float(np.median(bd)), 1), "sum_ms": round(float(bd.sum()) / 1e3, 2),
                       "what": "per wave batch of one ordered chain launch: the wave's lifetime (s_memrealtime); max = the "
                               "frame's critical path (one wave's chains), sum / launch time = mean resident waves"}
    chain_launches, chain_ms, chain_tests = stats[KERNEL_CHAIN]
    ch_launches, ch_ms, ch_tests = stats[KERNEL_CLOSEST_HIT]
    sh_launches, sh_ms, sh_tests = stats[KERNEL_SHADOW]
    _, shade_ms, _ = stats[KERNEL_SHADE]
    _, frame_ms, _ = stats[KERNEL_FRAME]
    bf = None
    if args.accel == "bvh" and not args.no_bf_roofline and rank == 0:
        scene.set_accel("brute_force")
        brun = main_run if world == 1 else Runner(1, frame_path=False)
        bst, _ = profile(1, brun)
        # counted work: the stages each (query, triangle) test reached, in a separate counting pass
        # (k_closest_hit_stages), priced per stage (rt_kernels.hip kTestStageFlops)
        scene.reset_stats()
        scene.set_profiling(True, count_work=True)
        brun.render_once()
        torch.cuda.synchronize(dev)
        scene.set_profiling(False)
        stages = [int(x) for x in scene.diag_read(0, len(TEST_STAGE_FLOPS))]
        scene.set_accel("bvh")
        l, ms, tests = bst[KERNEL_CLOSEST_HIT]
        flops = sum(c * f for c, f in zip(stages, TEST_STAGE_FLOPS))
        t = flops / (ms / 1e3) / 1e12
        bf = {"kernel": "k_closest_hit (brute force, --accel brute_force)", "bound": "valu",
              "achieved": round(t, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(t / FP32_PEAK_TFLOPS, 4),
              "peak_no_fma_no_pack": FP32_NOFMA_NOPACK_TFLOPS, "frac_no_fma_no_pack": round(t / FP32_NOFMA_NOPACK_TFLOPS, 4),
              "flop_per_launch": round(flops / max(l, 1)), "tests_per_launch": round(stages[0] / max(l, 1)),
              "stages_reached": stages, "flop_per_stage": list(TEST_STAGE_FLOPS),
              "work_what": "counted: per (query, triangle) test, the stages of rayIntersectTriangle it reached (plane "
                           "terms 14, division 1, in-plane coordinates and s 23, t 5, distance 9 flop; a test that "
                           "returns early is priced at the stages it ran), from a counting pass of the same frame",
              "note": "parity forbids FMA contraction (the x86 reference has none), so the packed-FMA peak is "
                      "unreachable; the no-FMA, non-packed issue rate is the practical ceiling",
              "launches": l, "avg_launch_ms": round(ms / max(l, 1), 3), "frame_closest_hit_ms": round(ms, 3)}

    result = None
    if rank == 0:
        total_rays = timed_rays if timed_rays else rays_per_step * args.steps
        value = total_rays / elapsed / 1e6
        queries = ch_tests / max(nt, 1)
        per_rank_steps = args.profile_steps * (fpc if main_run.single else kstep)   # frames (of steps) in the profiled launches
        traffic = traffic_src = None
        if args.accel == "bvh" and chain_launches > 0:
            # The chain kernel (every step of every sample per lane, RT_TUNE_CHAIN_FROM 0). Roof:
            # FP32 VALU at 37 flop per ray-triangle test and 52 per four-wide node
            # visit (device work counters). Logical (L1-side) bytes: 32 B per primary query in, a
            # 32-B chain record per closest-hit query, 64 B per node visit and per triangle test.
            kname = "k_chain"
            ch_launches, ch_ms = chain_launches, chain_ms   # the roofline's kernel from here on
            queries = rays_by_kind[0] / world * per_rank_steps
            tests_all, visits_all = bvh_tests + sh_bvh_tests, bvh_visits + sh_bvh_visits
            flops = tests_all * FLOP_PER_TEST + visits_all * FLOP_PER_NODE
            logical = (queries * 32.0 + (rays_by_kind[0] + rays_by_kind[1]) / world * per_rank_steps * 32.0 +
                       (visits_all + tests_all) * 64.0)
            bvh_tests, bvh_visits = tests_all, visits_all
            ch_tests = chain_tests
        elif args.accel == "bvh":
            kname = "k_bvh_closest_hit"
            flops = bvh_tests * FLOP_PER_TEST + bvh_visits * FLOP_PER_NODE
            logical = queries * 52.0 + (bvh_visits + bvh_tests) * 64.0
        else:
            kname = "k_closest_hit"
            flops = ch_tests * FLOP_PER_TEST
            logical = ch_tests / 64.0 * 64.0 + queries * 52.0
        avg_s = ch_ms / 1e3 / max(ch_launches, 1)
        achieved = flops / max(ch_launches, 1) / avg_s / 1e12 if avg_s > 0 else 0.0
        # the committed PMC summaries: profiles/*_pmc.json profiles the default workload (C4),
        # profiles/*_pmc_<workload>.json another one (tools/gpu_pmc.sh with WORKLOAD set)
        issue = None
        if args.accel == "bvh":
            traffic, traffic_src = pmc_traffic(kname, args.workload, multi=fpc > 1)
            pc, pc_src = pmc_counters(kname, "SQ_THREAD_CYCLES_VALU_per_launch", args.workload, multi=fpc > 1)
            if pc and avg_s > 0 and pc.get("SQ_INSTS_VALU_per_launch") and pc.get("SQ_ACTIVE_INST_VALU_per_launch"):
                simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
                iv = pc["SQ_INSTS_VALU_per_launch"]
                issue = {"valu_wave_instructions_per_launch": round(iv),
                         "valu_busy_frac": round(iv * VALU_CYCLES_PER_WAVE_INST / (simds * avg_s * CLOCK_HZ), 3),
                         "lane_utilization": round(pc["SQ_THREAD_CYCLES_VALU_per_launch"] /
                                                   (64.0 * pc["SQ_ACTIVE_INST_VALU_per_launch"]), 3),
                         "source": pc_src,
                         "what": "VALU issue roof: wave-instructions x 4 cycles (wave64, non-packed, "
                                 "profiles/r02_valu_rate.txt) / (SIMDs x launch time x 2.4 GHz); lane_utilization = "
                                 "SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU), the share of lanes active "
                                 "per issued VALU instruction"}
        rocprof = None
        if args.accel == "bvh":   # the same kernel's mean in the committed rocprof run (cross-check of avg_launch_ms)
            rp, rp_src = rocprof_mean(kname, args.workload, multi=fpc > 1)
            if rp and rp["mean_us"] > 0:
                ach = flops / max(ch_launches, 1) / (rp["mean_us"] * 1e-6) / 1e12
                rocprof = dict(rp, source=rp_src, achieved=round(ach, 3), frac=round(ach / FP32_PEAK_TFLOPS, 4),
                               what="the same work per launch over the rocprofv3 --kernel-trace mean of the committed "
                                    "profile (one frame in flight, launches after the first three)")
        dram = None
        if traffic and avg_s > 0:
            dram = {"achieved": round(traffic / avg_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(traffic / avg_s / 1e9 / HBM_PEAK_GBS, 4),
                    "bytes_per_launch": traffic, "source": traffic_src,
                    "what": "bytes past the XCD L2s (PMC 2*FETCH_SIZE + WRITE_SIZE, gfx950 correction) / "
                            "average launch time; Infinity Cache hits are included"}
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
                "frames_per_step": plan.frames // kstep,
                "steps_per_call": kstep if world > 1 else None,
                "width": WIDTH, "height": HEIGHT, "pf": PF, "max_lvl": MAX_LVL, "lights": [list(l) for l in LIGHTS],
                "triangles": nt, "vertices": nv, "tile": TILE,
                "parallelism": f"tile-shard{world}",
                "path": ("rt_render_frame_device" if main_run.single else
                         "rt_render_frames_sharded (library RCCL gather + un-permute)" if rtcomm is not None else
                         "rt_render_tiles_device + gloo host-staged gather (rehearsal) + rt_assemble_tiles_device"
                         if args.rehearse else
                         "rt_render_tiles_device + RCCL gather (torch.distributed) + rt_assemble_tiles_device"),
                "rays_per_step": int(rays_per_step),
                "rays_by_kind_per_step": {"primary": rays_by_kind[0], "secondary": rays_by_kind[1], "shadow": rays_by_kind[2]},
                "frame_ms_per_gpu": round(elapsed / args.steps * 1e3, 3),
                "frames_in_flight": inflight,
                "value_mode": value_mode,
                "value_mode_what": "value/ms_per_step come from the configured mode (--frames-per-call, --inflight); "
                                   "one_in_flight (and in_flight) time the same K frames in the other modes in the same run",
                "calibration_frames": calib,
                "calibration_what": "frames rendered one at a time before the warm-up, over the F pipelines of the "
                                    "timed mode in turn, until pipeline 0's launch trials were decided (rt_scene_trials; "
                                    "at most 64 per pipeline), then to the end of the round",
                "frames_in_flight_what": "consecutive frames of the view on alternating streams, each into its own "
                                         "buffer and fully rendered (RT_TUNE_FRAMES_IN_FLIGHT): a frame's launch starts "
                                         "while the previous frame's longest batches still run; ms_per_step is then "
                                         "the per-frame throughput time, one_in_flight the frame-after-frame time",
                "one_in_flight": one_in_flight,
                "in_flight": in_flight,
                "frames_per_call": fpc,
                "frames_per_call_what": "frames rendered by one rt_render_frames_device call: one chain launch whose wave "
                                        "tasks cycle over the frames (the frames overlap on one stream and one hardware "
                                        "queue); with camera_path, consecutive distinct views of the path; ms_per_step = "
                                        "wall clock / frames",
                "camera_path": path_what,
                "orbit": orbit,
                "multi_frame": multi_frame,
                "first_frame_ms": round(cold_ms, 3) if cold_ms is not None else None,
                "first_frame_what": "a new view's first frame (no measured batch order or launch trial: every order "
                                    "forgotten first), dispatched centre-out (RT_TUNE_COLD_ESTIMATE 2) as dynamic "
                                    "wave tasks (RT_TUNE_CHAIN_SPLIT 5), median of 3, host wall clock from the call to its render stream's completion (the library's background re-sort for the next frame not waited for)",
                "launch_trials": trials,
                "first_frame_screen_order_ms": round(cold_screen_ms, 3) if cold_screen_ms is not None else None,
                "scene_load_s": round(t_load, 3), "scene_gen_s": round(t_gen, 3),
            },
            "roofline": {
                "kernel": f"{kname} ({'every chain step: closest-hit, shadow and shade' if kname == 'k_chain' else 'primary + secondary queries'}, accel={args.accel})",
                "frames_per_launch": fpc,
                "bound": "valu",
                "achieved": round(achieved, 3),
                "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "traffic_unit": "bytes/launch (PMC: 2*FETCH_SIZE + WRITE_SIZE)",
                "flop_per_launch": round(flops / max(ch_launches, 1)),
                "flop_per_test": FLOP_PER_TEST,
                "flop_per_node_visit": FLOP_PER_NODE,
                "tests_per_launch": round((bvh_tests if args.accel == "bvh" else ch_tests) / max(ch_launches, 1)),
                "node_visits_per_launch": round(bvh_visits / max(ch_launches, 1)) if args.accel == "bvh" else 0,
                "queries_per_launch": round(queries / max(ch_launches, 1)),
                "launches": ch_launches,
                "avg_launch_ms": round(avg_s * 1e3, 4),
                "timing": f"HIP events on the launch stream, mean over {args.profile_steps} batch-ordered launches of the timed "
                          f"entry point, one frame in flight",
                "rocprof": rocprof,
                "dram": dram,
                "issue": issue,
                "logical_bytes_per_launch": round(logical / max(ch_launches, 1)),
                "logical_bytes_what": "L1-side accesses (64 B per node visit and per triangle test, 32 B per query "
                                      "in and per chain record out); most are served by L1/L2, so this is not HBM traffic",
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
            "batches": batches,
            "accel": {"mode": args.accel, "bvh": bvh_info},
            "cpu_baseline": None,
        }
        result.update(extra)
        if shares is not None:
            result["strong_shares"] = dict(shares, what="rank r's 1/N share of ONE frame (rt_render_tiles_device, tiles r, "
                                           "r + N, ...), every rank, rendered on this GPU after its batch order and launch "
                                           "trials settled: ms = median launch, one at a time (HIP events); max_ms = the "
                                           "slowest rank (the frame time at N before the gather); pipelined_ms = four frames' "
                                           "shares per call, calls back to back, per frame; assemble_ms = rank 0's device "
                                           "un-permute of N shards; max_batch_us = the share's longest wave batch")
        if e2e is not None:
            result["config"]["end_to_end"] = e2e
        if world == 1 and batches:
            result["strong_model"] = strong_model((one_in_flight or {}).get("ms_per_step") or elapsed / args.steps * 1e3,
                                                  batches["max_us"] / 1e3, extra.get("shard_path", {}).get("ms_per_step"),
                                                  WIDTH * HEIGHT * 3, shares=shares, t1_pipe_ms=elapsed / args.steps * 1e3)
        if rehearsal is not None:
            result["rehearsal"] = rehearsal
        if args.ppm and timed_last is not None:
            R.write_ppm(args.ppm, timed_last[0].cpu().numpy())

    # ---- the reference's own caller unchanged: main.cpp's 'r' loop over the source-level drop-in ----
    if rank == 0 and world == 1 and wl.get("dropin") and not args.no_dropin:
        result["dropin_loop"] = dropin_loop(obj, wl)

    # ---- CPU baseline + in-run parity on a bounded tile sample (rank 0, N=1 only) ----
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(obj, params, timed_last[0].cpu().numpy(), layout, args, wl, corners=timed_corners)
        result["cpu_baseline"]["parity_vs_gpu"]["frame"] = timed_last_what
        if orbit_last is not None:   # the last timed orbit view, on tiles across its sphere region
            result["config"]["orbit"]["parity_vs_cpu"] = orbit_parity(obj, params, orbit_last, wl)

    if rtcomm is not None:
        rtcomm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


def multiframe_leg(scene, run, cparams, W, H, args, rays_per_frame, dev):
    """rt_render_frames_device: K frames of the view in one chain launch (K = 2, 4), one call at a time
    on one stream, and K = 2 with two calls in flight (RT_TUNE_FRAMES_IN_FLIGHT 2, two streams). Every
    frame is fully rendered; ms_per_frame = wall clock / frames."""
    import torch
    K_MAX = 8
    bufs = [torch.zeros(H * W * 3, dtype=torch.uint8, device=dev) for _ in range(2 * K_MAX)]
    out = {"what": "K frames of the SAME (default) view per rt_render_frames_device call (one chain launch whose wave "
                   "tasks cycle over the frames), calls back to back; every frame fully rendered (identical copies: the "
                   "headline's calls render distinct camera-path views instead)"}
    for K, fif in ((2, 1), (4, 1), (8, 1), (2, 2), (4, 2)):
        scene.tune("frames_in_flight", fif)
        calls = max(max(args.steps, LEG_STEPS) // K, 2)

        def call(i):
            st = run.fstreams[i % fif] if fif <= len(run.fstreams) else run.fstreams[0]
            base = (i % 2) * K
            scene.render_frames_device([cparams] * K, TILE, TILE, [b.data_ptr() for b in bufs[base:base + K]], bufs[0].numel(),
                                       st.cuda_stream)
        for i in range(max(args.warmup, 2) * fif):
            call(i)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(calls):
            call(i)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        frames = calls * K
        out[f"k{K}_inflight{fif}"] = {"frames": frames, "ms_per_frame": round(el / frames * 1e3, 4),
                                      "value": round(rays_per_frame * frames / el / 1e6, 4)}
    scene.tune("frames_in_flight", 1)
    return out


def orbit_leg(scene, run, W, H, PF, MAX_LVL, LIGHTS, flags, args, inflight, obj, dev):
    """A moving view: frame i renders view i of an orbit (scenes.orbit_corners: the default view turned
    by i * --orbit-step degrees about the world y axis, the trackball's effect on produceRay's corner
    rays; MyCameraPosition fixed, main.cpp:222), so no two frames share a view. Warm-up frames are new
    views too; the batch order and launch trials carry over from view to view (their key is the frame
    geometry). Timed with the static leg's frames in flight and one at a time, every frame fully
    rendered; rays are counted per view afterwards (each view has its own count). The last timed
    frame is kept for the in-run oracle check (cpu_baseline)."""
    import torch

    import raytracert_amd as R
    from raytracert_amd import scenes
    warm, K = max(args.warmup, 2) * inflight, max(args.steps, LEG_STEPS)
    fpc = args.frames_per_call if not args.no_multi_frame else 1
    calls = max(K // fpc, 1)
    # (enough views for the multi-frame calls below too: at small --steps a call holds more views than K)
    nviews = max(warm + K, warm + calls * fpc, max(warm // fpc, 2) * fpc) if fpc > 1 else warm + K
    corners = [scenes.orbit_corners(W, H, k + 1, args.orbit_step) for k in range(nviews)]
    views = [R.RenderParams(width=W, height=H, pf=PF, max_lvl=MAX_LVL, lights=LIGHTS, flags=flags, corners=c).to_c()
             for c in corners]

    def loop(fif, first, n):
        scene.tune("frames_in_flight", fif)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(n):
            fb, st = run.fbufs[i % max(2, fif)], run.fstreams[i % fif]
            scene.render_frame_device(views[first + i], TILE, TILE, fb.data_ptr(), fb.numel(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    loop(inflight, 0, warm)
    el = loop(inflight, warm, K)
    last = run.fbufs[(K - 1) % max(2, inflight)].clone().view(H, W, 3)
    torch.cuda.synchronize(dev)
    el1 = loop(1, warm, K) if inflight > 1 else el
    # a camera path rendered --frames-per-call consecutive views per rt_render_frames_device call (one
    # chain launch over the views, one call at a time); the call's last view re-rendered alone must match
    multi = None
    if fpc > 1:
        scene.tune("frames_in_flight", 1)
        st = run.fstreams[0]

        def mcall(first, i):
            bufs = run.fbufs[(i % 2) * fpc:(i % 2) * fpc + fpc]
            scene.render_frames_device(views[first + i * fpc:first + i * fpc + fpc], TILE, TILE,
                                       [b.data_ptr() for b in bufs], bufs[0].numel(), st.cuda_stream)
            return bufs[-1]
        for i in range(max(warm // fpc, 2)):
            mcall(0, i)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(calls):
            lastb = mcall(warm, i)
        torch.cuda.synchronize(dev)
        elm = time.perf_counter() - t0
        alone = torch.zeros_like(lastb)
        scene.render_frame_device(views[warm + calls * fpc - 1], TILE, TILE, alone.data_ptr(), alone.numel(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        multi = {"frames_per_call": fpc, "views_timed": calls * fpc, "ms_per_step": round(elm / (calls * fpc) * 1e3, 3),
                 "last_view_equals_alone": bool(torch.equal(lastb, alone))}
    rays = 0
    for k in range(warm, warm + K):
        fb = run.fbufs[0]
        c = scene.render_frame_device(views[k], TILE, TILE, fb.data_ptr(), fb.numel(), run.fstreams[0].cuda_stream,
                                      want_counts=True)
        rays += int(sum(int(x) for x in c))
    scene.tune("frames_in_flight", 1)
    return {"what": f"every frame a new view: the default view turned by frame x {args.orbit_step} degrees about the "
                    f"world y axis (the trackball, then 'r'), {warm} warm-up and {K} timed views, each fully rendered; "
                    f"order and launch trials carried over from view to view",
            "step_deg": args.orbit_step, "views_timed": K, "first_timed_deg": round((warm + 1) * args.orbit_step, 3),
            "frames_in_flight": inflight,
            "ms_per_step": round(el / K * 1e3, 3), "value": round(rays / el / 1e6, 4),
            "one_in_flight": {"ms_per_step": round(el1 / K * 1e3, 3), "value": round(rays / el1 / 1e6, 4)},
            "views_per_call": (dict(multi, value=round(rays / K / (elm / multi["views_timed"]) / 1e6, 4)) if multi else None),
            "rays_per_frame_mean": round(rays / K), "unit": "Mrays/s",
            "_last": (last, corners[warm + K - 1])}


def strong_shares(scene, cparams, W, H, dev, ns=(2, 4, 8), reps=15, warm=12, pipelined_k=4, ranks=None):
    """Strong scaling measured on one GPU: for N = 2/4/8, rank r's 1/N share of ONE frame
    (rt_render_tiles_device, first = r, stride = N: what rank r renders when one frame is split over N
    GPUs, main.cpp:369-395 has no cross-pixel state) is rendered on its own until its batch order and
    launch trials have settled, then timed launch by launch (HIP events on the launch stream, each
    launch synchronised: one frame's latency) and back to back (`pipelined_k` frames' shares per call:
    a stream of frames). The frame time at N is bound by the slowest rank: `max_ms` over the ranks.
    The device un-permute of N shards into the frame (rt_assemble_tiles_device) is timed the same way.
    Returns a dict keyed n2/n4/n8."""
    import numpy as np
    import torch

    import raytracert_amd as R
    from raytracert_amd import dist as rdist
    st = torch.cuda.current_stream(dev)
    layout = rdist.TileLayout(W, H, TILE, TILE)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed_launch(fn):
        ev[0].record(st)
        fn()
        ev[1].record(st)
        torch.cuda.synchronize(dev)
        return ev[0].elapsed_time(ev[1])

    out = {}
    for N in ns:
        per_rank = []
        plan_k = rdist.ShardPlan(layout, N, frames=pipelined_k)
        buf = torch.zeros(max(layout.shard_bytes(N), plan_k.shard_bytes), dtype=torch.uint8, device=dev)
        for r in (range(N) if ranks is None else [x for x in ranks if x < N]):
            def call(k=1):
                scene.render_tiles_device(cparams, TILE, TILE, r, N, buf.data_ptr(), buf.numel(), st.cuda_stream, frames=k)
            call()   # (a new batch geometry: its first launch resets the trials trials() reports)
            torch.cuda.synchronize(dev)
            n = 1
            while n < 64 and scene.trials()["choice"] < 0:   # (the share's own launch trials: as calibrate())
                call()
                torch.cuda.synchronize(dev)
                n += 1
            for _ in range(warm):
                call()
            torch.cuda.synchronize(dev)
            lat = sorted(timed_launch(call) for _ in range(reps))
            bd = scene.batch_durations()
            tr = scene.trials()
            # pipelined: pipelined_k frames' shares per call (one launch), calls back to back
            call(pipelined_k)
            torch.cuda.synchronize(dev)
            m = 1
            while m < 64 and scene.trials()["choice"] < 0:
                call(pipelined_k)
                torch.cuda.synchronize(dev)
                m += 1
            for _ in range(3):
                call(pipelined_k)
            torch.cuda.synchronize(dev)
            ev[0].record(st)
            for _ in range(reps):
                call(pipelined_k)
            ev[1].record(st)
            torch.cuda.synchronize(dev)
            pip = ev[0].elapsed_time(ev[1]) / reps / pipelined_k
            per_rank.append({"rank": r, "tiles": layout.tiles_of(r, N), "ms": round(lat[len(lat) // 2], 4),
                             "min_ms": round(lat[0], 4), "pipelined_ms": round(pip, 4),
                             "max_batch_us": round(float(bd.max()), 1) if bd.size else None,
                             "batches": int(bd.size), "calib": n, "choice": tr["choice"], "steal": tr["wave_steal"],
                             "dist": tr["chain_split"]})
        # the un-permute of N one-frame shards on rank 0 (the bytes do not change its time)
        gathered = torch.zeros(N * layout.shard_bytes(N), dtype=torch.uint8, device=dev)
        frame = torch.zeros(H * W * 3, dtype=torch.uint8, device=dev)

        def assemble():
            R.assemble_tiles_device(dev.index or 0, W, H, TILE, TILE, 1, N, gathered.data_ptr(), gathered.numel(),
                                    frame.data_ptr(), frame.numel(), st.cuda_stream)
        assemble()
        asm = sorted(timed_launch(assemble) for _ in range(reps))[reps // 2]
        worst = max(per_rank, key=lambda d: d["ms"])
        out[f"n{N}"] = {"max_ms": worst["ms"], "max_rank": worst["rank"],
                        "mean_ms": round(float(np.mean([d["ms"] for d in per_rank])), 4),
                        "pipelined_max_ms": max(d["pipelined_ms"] for d in per_rank),
                        "assemble_ms": round(asm, 4), "ranks": per_rank}
    return out


def end_to_end(scene, cparams, W, H, dev, frames=40, threads=8, workdir=None, inflight=2):
    """A frame as the reference's 'r' key ends it (main.cpp:347-405): the render, the bytes in host
    memory (Image::_image's quantised bytes; here one device-to-host copy of the uint8 frame into pinned
    memory), then writeImage("result.ppm") (rt_ppm_writer: the file kept mapped, `threads` threads copy
    the frame in; the same file as rt_write_ppm, which is timed beside it). Two modes over `frames` frames:
    one at a time (render, copy, write in sequence, each synchronised) and pipelined (frame i's copy on
    a copy stream and its PPM write on the host overlap frame i + 1's render, the renders `inflight`
    frames in flight on alternating streams, RT_TUNE_FRAMES_IN_FLIGHT). Host wall clock."""
    import numpy as np
    import torch

    import raytracert_amd as R
    st = torch.cuda.current_stream(dev)
    cs = torch.cuda.Stream(dev)
    rs = [st] + [torch.cuda.Stream(dev) for _ in range(max(1, inflight) - 1)]   # render streams
    n = H * W * 3
    fbs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(2)]
    hbs = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    path = os.path.join(workdir or tempfile.mkdtemp(prefix="rt_e2e_"), "result.ppm")
    path1 = os.path.join(os.path.dirname(path), "result_fwrite.ppm")
    writer = R.PpmWriter(path, W, H, threads)
    ev_r = [torch.cuda.Event() for _ in range(2)]
    ev_c = [torch.cuda.Event() for _ in range(2)]

    def render(i, k=1):
        s_ = rs[i % k]
        scene.render_frame_device(cparams, TILE, TILE, fbs[i % 2].data_ptr(), n, s_.cuda_stream)
        ev_r[i % 2].record(s_)

    def copy(i):
        cs.wait_event(ev_r[i % 2])
        with torch.cuda.stream(cs):
            hbs[i % 2].copy_(fbs[i % 2], non_blocking=True)
        ev_c[i % 2].record(cs)

    def write(i):
        ev_c[i % 2].synchronize()
        writer.write_ptr(hbs[i % 2].data_ptr())

    # one at a time: each stage waits for the one before it (a host that renders, reads and saves)
    parts = {"render": [], "copy": [], "write": [], "write_fwrite": []}
    for i in range(frames + 3):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        render(i)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        copy(i)
        cs.synchronize()
        t2 = time.perf_counter()
        write(i)
        t3 = time.perf_counter()
        R.write_ppm(path1, hbs[i % 2].numpy().reshape(H, W, 3))   # (rt_write_ppm: fopen + fwrite, one thread)
        t4 = time.perf_counter()
        if i >= 3:
            for k, v in zip(parts, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                parts[k].append(v * 1e3)
    one = {k: round(float(np.median(v)), 4) for k, v in parts.items()}
    one["ms_per_frame"] = round(one["render"] + one["copy"] + one["write"], 4)
    # pipelined: frame i's copy and write overlap frame i + 1's render
    def pipelined(count):
        k = len(rs)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(count):
            if i >= 2:
                rs[i % k].wait_event(ev_c[i % 2])   # (frame i reuses frame i - 2's device buffer)
            render(i, k)
            copy(i)
            if i >= 1:
                write(i - 1)
        write(count - 1)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0
    if len(rs) > 1:
        scene.tune("frames_in_flight", len(rs))
    pipelined(4 * len(rs))
    runs = sorted(pipelined(frames) for _ in range(3))   # (the median of three runs: a run is ~20 ms of host work)
    el = runs[1]
    scene.tune("frames_in_flight", 1)
    writer.close()
    with open(path, "rb") as f:   # the last frame's file is the last frame's bytes
        body = f.read()
    ok = body[:len(f"P6\n{W} {H}\n255\n")] == f"P6\n{W} {H}\n255\n".encode() and \
        np.array_equal(np.frombuffer(body, np.uint8, offset=len(body) - n), fbs[(frames - 1) % 2].cpu().numpy())
    return {"what": "render -> uint8 frame in host memory (pinned, one device-to-host copy) -> result.ppm "
                    "(rt_ppm_writer: the file kept mapped, the frame copied in by ppm_threads threads; write_fwrite = "
                    "rt_write_ppm, fopen + fwrite, for comparison), as main.cpp:347-405 ends a frame; host wall clock, "
                    "medians",
            "frames": frames, "ppm_threads": threads, "one_at_a_time": one,
            "pipelined": {"ms_per_frame": round(el / frames * 1e3, 4), "renders_in_flight": len(rs),
                          "runs_ms_per_frame": [round(x / frames * 1e3, 4) for x in runs],
                          "what": "frame i's copy (copy stream) and PPM write (host) overlap frame i + 1's render; "
                                  "consecutive renders on alternating streams (RT_TUNE_FRAMES_IN_FLIGHT)"},
            "last_file_equals_frame": bool(ok)}


def strong_model(t1_ms, crit_ms, shard_ms, frame_bytes, link_gbs=(50.0, 150.0), rccl_lat_ms=0.02, sync_ms=0.02, shares=None,
                 t1_pipe_ms=None):
    """Per-frame time of ONE frame split over N GPUs (strong scaling). With `shares`
    (strong_shares, r06: every rank's 1/N share of the frame rendered and timed on this GPU) the
    render is the slowest rank's measured share and the un-permute its measured time; without, the
    r04 model: max(t1 / N, the frame's longest wave batch) and the shard path minus the frame path.
    The gather stays a model (one GPU here): rank 0 receives frame_bytes / N from each peer on its
    own xGMI link at an assumed 50-150 GB/s, plus a collective latency, then a barrier.
    Two readings: `latency` is one frame on its own (render, then gather, un-permute and barrier in
    sequence); `pipelined` is the frame rate of a stream of frames (bench.py's --mode strong: step i's
    gather and un-permute overlap step i + 1's render; measured shares: four frames' shares per render
    call), the slowest stage plus the barrier. Speedups: latency against t1_ms (one frame at a time on
    one GPU), pipelined against t1_pipe_ms (the one-GPU frame rate of the timed loop; default t1_ms)."""
    t1p = t1_pipe_ms or t1_ms
    assemble_ms = max(0.0, (shard_ms or t1_ms) - t1_ms)
    out = {"inputs": {"t1_ms": round(t1_ms, 4), "t1_pipelined_ms": round(t1p, 4), "critical_path_ms": round(crit_ms, 4), "assemble_ms": round(assemble_ms, 4),
                      "frame_bytes": frame_bytes, "link_gbs": list(link_gbs), "rccl_latency_ms": rccl_lat_ms,
                      "sync_ms": sync_ms, "render": "measured shares (strong_shares)" if shares else "modelled"}}
    for n in (2, 4, 8):
        sh = (shares or {}).get(f"n{n}")
        if sh:
            render, render_p, asm = sh["max_ms"], sh["pipelined_max_ms"], sh["assemble_ms"]
            bound = "measured: the slowest rank's share"
        else:
            render = render_p = max(t1_ms / n, crit_ms)
            asm = assemble_ms
            bound = "critical path" if crit_ms >= t1_ms / n else "work / N"
        res = {}
        for bw in link_gbs:
            gather = frame_bytes / n / (bw * 1e9) * 1e3 + rccl_lat_ms
            t = render + gather + asm + sync_ms
            tp = max(render_p, gather, asm) + sync_ms
            res[f"{int(bw)}GBs"] = {"latency_ms_per_frame": round(t, 4), "latency_speedup": round(t1_ms / t, 2),
                                    "pipelined_ms_per_frame": round(tp, 4), "pipelined_speedup": round(t1p / tp, 2)}
        out[f"n{n}"] = {"render_ms": round(render, 4), "render_pipelined_ms": round(render_p, 4), "assemble_ms": round(asm, 4),
                        "bound": bound, **res}
    return out


def timed_instantiation(kernel: str, name: str, multi: bool) -> bool:
    """Whether profiled kernel `name` is the timed loop's instantiation of `kernel`: for k_chain<W,
    kAnyHit, kCount, kInLane, kSteal, kQuad, kMulti>, not the counting one (kCount false), and the
    multi-frame one (kMulti) exactly when the timed loop renders several frames per call (older
    profiles, before kQuad/kMulti: any non-counting one)."""
    if name == kernel:
        return True
    if not name.startswith(kernel + "<"):
        return False
    targs = [a.strip() for a in name[name.index("<") + 1:name.rindex(">")].split(",")]
    if kernel != "k_chain":
        return targs[-1] == "false"
    if len(targs) > 2 and targs[2] != "false":
        return False
    return len(targs) < 7 or targs[6] == ("true" if multi else "false")


def profile_age(path: str):
    """Sort key of a round-tagged profile name, oldest first: r06z_pmc.json < r06aa_pmc.json (a round's
    tags run a..z, then aa, ab, ...; a plain string sort would put r06z after r06aa)."""
    import re
    m = re.match(r"r(\d+)([a-z0-9]*?)_", os.path.basename(path))
    if not m:
        return (-1, 0, os.path.basename(path))
    tag = re.match(r"[a-z]*", m.group(2)).group(0)
    return (int(m.group(1)), len(tag), m.group(2))


def rocprof_mean(kernel: str, workload: str = "c4", multi: bool = False):
    """The committed rocprofv3 kernel-trace summary of `kernel` (tools/kernel_trace_summary.py over
    tools/gpu_final.sh's rocprof run of this bench, one frame in flight): the instantiation with the
    most launches, its mean duration after the first three launches. (dict, file) or (None, None)."""
    import glob
    if workload != "c4":
        return None, None
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*_kernel_trace_summary.json")), key=profile_age, reverse=True):
        try:
            ks = json.load(open(f)).get("kernels", {})
        except (OSError, ValueError):
            continue
        names = [n for n in ks if timed_instantiation(kernel, n, multi)]
        if names:
            n = max(names, key=lambda k: ks[k].get("launches", 0))
            return {"instantiation": n, "launches": ks[n]["launches"], "mean_us": ks[n].get("mean_after_first_3_us", ks[n]["mean_us"])}, \
                os.path.relpath(f, HERE)
    return None, None


def pmc_traffic(kernel: str, workload: str = "c4", multi: bool = False):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary of `workload`
    (profiles/*_pmc.json for C4, profiles/*_pmc_<workload>.json otherwise; written by
    tools/pmc_summary.py from separate rocprofv3 --pmc passes of this bench command)."""
    c, src = pmc_counters(kernel, "traffic_bytes_per_launch", workload, multi)
    return (c["traffic_bytes_per_launch"], src) if c else (None, None)


def pmc_counters(kernel: str, need: str, workload: str = "c4", multi: bool = False):
    """The per-launch counters of `kernel` (its timed instantiation) from the newest committed PMC
    summary of `workload` that has counter `need`: (dict, file) or (None, None)."""
    import glob
    suffix = "_pmc.json" if workload == "c4" else f"_pmc_{workload}.json"
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "*" + suffix)), key=profile_age)   # oldest first
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        ks = d.get("kernels", {})
        # the timed loop's instantiation of the kernel (timed_instantiation)
        names = [n for n in ks if timed_instantiation(kernel, n, multi)]
        names.sort(key=lambda n: -ks[n].get("launches_in_pass", 0))
        for n in names:
            if need in ks[n]:
                return ks[n], os.path.relpath(f, HERE)
    return None, None


def dropin_loop(obj, wl):
    """main.cpp's 'r' key as written (one performRayTracing per sub-sample, then RGBValue and
    Image::writeImage) compiled against include/raytracert_dropin.hpp: tests/cxx/dropin_main.cpp built
    with g++ here, run as a child process on the same GPU. Times the literal loop (the drop-in answers
    its sub-samples from one frame-wide trace), the one-call renderImage(), and single
    performRayTracing calls on rays of no frame (the per-call round trip)."""
    import subprocess
    d = tempfile.mkdtemp(prefix="rt_dropin_")
    exe = os.path.join(d, "dropin_main")
    lib = os.path.join(HERE, "raytracert_amd")
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-I" + os.path.join(HERE, "include"),
                    os.path.join(HERE, "tests", "cxx", "dropin_main.cpp"), "-L" + lib, "-lrtamd", "-Wl,-rpath," + lib,
                    "-o", exe], check=True)
    # ref_default: pf stays the reference's default 3 and max_lvl its 10 (the drop-in's globals); other
    # workloads set theirs with the host's keys first (C4: '-' twice for pf 1, max_lvl 3, the second
    # light); 'T' x2: the first frame includes the upload of the workspace; 'V:200' checks 200 of the
    # frame's cached colours against the per-call path (trace() of the loop's own ray), bit for bit
    keys = list(wl.get("dropin_keys", ())) + ["T", "T", "V:200", "R", "P:2000", "H", "H"]
    out = subprocess.run([exe, "keys", obj, str(wl["width"]), str(wl["height"]), os.path.join(d, "f")] + keys,
                         check=True, capture_output=True, text=True, timeout=600).stdout.splitlines()
    fr = [l.split() for l in out if l.startswith("frame ")]
    single = next(l.split() for l in out if l.startswith("single "))
    floor = [float(l.split()[7]) for l in out if l.startswith("hostfloor ")]
    loop_ms = float(fr[1][10])
    n = wl["width"] * wl["height"] * wl["pf"] ** 2
    ver = next((l.split() for l in out if l.startswith("verify ")), None)
    return {"what": "main.cpp:355-395 unchanged (performRayTracing per sub-sample) over the drop-in header, "
                    f"{wl['width']}x{wl['height']} pf {wl['pf']} = {n} calls",
            "loop_ms": loop_ms, "first_loop_ms": float(fr[0][10]), "render_image_ms": float(fr[2][7]),
            "frame_trace_ms": float(fr[1][12]), "first_frame_trace_ms": float(fr[0][12]),
            "frame_trace_what": "the loop's first performRayTracing call, which traces the whole frame on the GPU "
                                "(rt_trace_frame_samples) and copies every sub-sample's ray and colour to pinned host memory",
            "host_floor_ms": min(floor) if floor else None,
            "host_floor_what": "the same loop with performRayTracing replaced by a function that only reads its "
                               "arguments: the unchanged loop's own cost (two divisions and ~60 flops per call)",
            "single_call_us": float(single[4]), "single_calls": int(single[1]),
            "per_call_loop_estimate_s": round(float(single[4]) * n / 1e6, 1),
            "frames_equal": open(fr[1][1], "rb").read() == open(fr[2][1], "rb").read(),
            "keys": keys,
            "cached_vs_per_call": ({"records": int(ver[1]), "ray_diff": int(ver[4]), "rgb_diff": int(ver[6])} if ver else None)}


def host_cpu():
    """The host the CPU baseline ran on: logical CPUs, this process's CPU share, CPU model."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        share = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        share = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity": share, "model": model or "unknown"}


def orbit_parity(obj, params, last, wl):
    """The in-run parity check of the orbit leg: tiles of its last timed view against the CPU
    restatement at that view's corner rays (the cpu_baseline leg's checker)."""
    import numpy as np
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle as O
    frame, corners = last
    img = frame.cpu().numpy()
    op = O.make_params(params.width, params.height, params.pf, params.max_lvl, lights=params.lights, flags=params.flags,
                       seed=params.seed, corners=corners)
    sc = O.OracleScene(obj)
    w, h = params.width, params.height
    tiles = [((w // 2 // TILE + dx) * TILE, (h // 2 // TILE + dy) * TILE) for dx, dy in ((0, 0), (-12, -8), (12, 8), (-20, 10))]
    exact = total = max_d = 0
    for x0, y0 in tiles:
        _, u8, _ = sc.render(op, x0, y0, TILE, TILE, nthreads=16)
        d = np.abs(img[y0:y0 + TILE, x0:x0 + TILE].astype(np.int16) - u8.astype(np.int16))
        max_d, exact, total = max(max_d, int(d.max())), exact + int((d == 0).sum()), total + d.size
    return {"tiles": tiles, "bytes": total, "exact_frac": round(exact / max(total, 1), 6), "max_lsb": max_d,
            "frame": "the last timed orbit view"}


def cpu_baseline(obj, params, gpu_frame, layout, args, wl, corners=None):
    """Time the CPU restatement (oracle/, 'port') on every k-th 16x16 tile of the same frame (C2:
    the whole frame) with --cpu-threads threads, and on every --cpu-single-every-th of those tiles
    with one thread; check the GPU's bytes on the sampled tiles against it."""
    import numpy as np
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle as O
    sc = O.OracleScene(obj)
    op = O.make_params(params.width, params.height, params.pf, params.max_lvl, lights=params.lights, flags=params.flags,
                       seed=params.seed, corners=corners)   # (corners: the checked frame's view; None = the default)
    every = args.cpu_sample_every or wl.get("cpu_every", 96)
    threads = args.cpu_threads

    def rects(tiles):
        for t in tiles:
            ty, tx = divmod(t, layout.tiles_x)
            x0, y0 = tx * layout.tile_w, ty * layout.tile_h
            yield x0, y0, min(layout.tile_w, params.width - x0), min(layout.tile_h, params.height - y0)

    def run(rs, nthreads):
        rays, outs = 0, []
        t0 = time.perf_counter()
        for x0, y0, w, h in rs:
            _, u8, c = sc.render(op, x0, y0, w, h, nthreads=nthreads)
            rays += int(c.sum())
            outs.append((x0, y0, w, h, u8))
        return rays, time.perf_counter() - t0, outs

    if every == 1:   # the whole frame in one call (row-interleaved threads)
        rays, dt, outs = run([(0, 0, params.width, params.height)], threads)
        what = f"the whole {params.width}x{params.height} frame"
        tiles = list(range(0, layout.n_tiles, 97))
    else:
        tiles = list(range(0, layout.n_tiles, every))
        rays, dt, outs = run(rects(tiles), threads)
        what = f"{len(tiles)} of {layout.n_tiles} 16x16 tiles (every {every}th)"
    # one thread: 4x4-pixel blocks at the sampled tiles' corners until the time budget is spent
    rays1, dt1, blocks = 0, 0.0, 0
    for x0, y0, w, h in rects(tiles):
        r, d, _ = run([(x0, y0, min(w, 4), min(h, 4))], 1)
        rays1, dt1, blocks = rays1 + r, dt1 + d, blocks + 1
        if dt1 >= args.cpu_single_budget:
            break
    max_d = exact = total = 0
    for x0, y0, w, h, u8 in outs:
        g = gpu_frame[y0:y0 + h, x0:x0 + w]
        d = np.abs(g.astype(np.int16) - u8.astype(np.int16))
        max_d = max(max_d, int(d.max()))
        exact += int((d == 0).sum())
        total += d.size
    hc = host_cpu()
    return {
        "value": round(rays / dt / 1e6, 6),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{what} of the same {wl['desc'].split(':')[0]} frame, {rays} rays in {dt:.1f} s, "
                  f"oracle/rt_oracle.c (-O2, brute force) on {threads} threads",
        "single_thread": {"value": round(rays1 / dt1 / 1e6, 6), "unit": "Mrays/s", "cores": 1,
                          "sample": f"{blocks} 4x4-pixel blocks at sampled tiles, {rays1} rays in {dt1:.1f} s"},
        "host": hc,
        "host_note": f"{threads} threads = the GPU box's CPU share per GPU (nproc {hc['nproc']} counts the whole "
                     f"machine's CPUs, most of them not ours)",
        "parity_vs_gpu": {"bytes": total, "exact_frac": round(exact / max(total, 1), 6), "max_lsb": max_d},
    }


if __name__ == "__main__":
    main()
