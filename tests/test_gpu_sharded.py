"""The C-ABI multi-GPU path (rt_render_frames_sharded + rt_comm_*, rt_assemble_tiles_device;
SURVEY.md §8e) on the GPU: the interleaved shards of N simulated ranks, placed as one gather lays
them out and un-permuted by the library, equal the one-GPU frame for N = 2, 3, 5 and multi-frame
batches; a world-1 RCCL communicator renders through the real gather; with two or more GPUs
visible, two processes render one frame over RCCL."""
import os
import subprocess
import sys

import numpy as np
import pytest

import raytracert_amd as R
from _util import scene_path

pytestmark = pytest.mark.gpu

LIGHTS = [(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)]


def _frame(sc, p):
    import torch
    fb = torch.zeros(p.height * p.width * 3, dtype=torch.uint8, device="cuda:0")
    c = sc.render_frame_device(p, 16, 16, fb.data_ptr(), fb.numel(), torch.cuda.current_stream().cuda_stream,
                               want_counts=True)
    return fb.view(p.height, p.width, 3).cpu().numpy(), c


@pytest.mark.parametrize("nranks,frames,size,tile", [(2, 1, (100, 70), 16), (3, 2, (100, 70), 16), (5, 3, (61, 29), 8),
                                                     (3, 1, (1920, 1080), 16)])
def test_assemble_composes_interleaved_shards(nranks, frames, size, tile, workdir, gpu_available):
    import torch
    w, h = size
    p = R.RenderParams(width=w, height=h, pf=1, max_lvl=3, lights=LIGHTS)
    T = ((w + tile - 1) // tile) * ((h + tile - 1) // tile)
    slots = (frames * T + nranks - 1) // nranks
    shard = slots * tile * tile * 3
    stream = torch.cuda.current_stream().cuda_stream
    with R.Scene.load(scene_path("syn:C4" if w > 1000 else "syn:F3", workdir), device=0) as sc:
        full, c1 = _frame(sc, R.RenderParams(width=w, height=h, pf=1, max_lvl=3, lights=LIGHTS))
        gathered = torch.full((nranks * shard,), 9, dtype=torch.uint8, device="cuda:0")
        total = np.zeros(3, np.uint64)
        for r in range(nranks):   # what one gather of equal-sized shards lays out
            part = gathered[r * shard:(r + 1) * shard]
            n, c = sc.render_tiles_device(p, tile, tile, r, nranks, part.data_ptr(), part.numel(), stream,
                                          want_counts=True, frames=frames)
            assert n == (frames * T - r + nranks - 1) // nranks
            total += c
        out = torch.zeros(frames * h * w * 3, dtype=torch.uint8, device="cuda:0")
        R.assemble_tiles_device(0, w, h, tile, tile, frames, nranks, gathered.data_ptr(), gathered.numel(), out.data_ptr(),
                                out.numel(), stream)
        frames_out = out.view(frames, h, w, 3).cpu().numpy()
    for f in range(frames):
        assert np.array_equal(frames_out[f], full), f
    assert [int(x) for x in total] == [frames * int(x) for x in c1]


def _unpermute_reference(gathered, w, h, tile, frames, nranks):
    """numpy restatement of the un-permute's layout: global tile g = f * T + t is held by rank g % N in
    slot g / N; each tile is tile x tile x 3 bytes, clipped at the frame's right and bottom edges."""
    tx_n, ty_n = (w + tile - 1) // tile, (h + tile - 1) // tile
    T = tx_n * ty_n
    slots = (frames * T + nranks - 1) // nranks
    tiles = gathered.reshape(nranks, slots, tile, tile, 3)
    out = np.zeros((frames, ty_n * tile, tx_n * tile, 3), np.uint8)
    for g in range(frames * T):
        f, t = divmod(g, T)
        ty, tx = divmod(t, tx_n)
        out[f, ty * tile:(ty + 1) * tile, tx * tile:(tx + 1) * tile] = tiles[g % nranks, g // nranks]
    return out[:, :h, :w]


@pytest.mark.parametrize("nranks,frames,size,tile,offset", [(3, 2, (176, 90), 16, 0), (8, 3, (800, 600), 16, 0),
                                                            (8, 2, (1920, 1080), 16, 0), (1, 1, (256, 32), 16, 0),
                                                            (7, 2, (800, 600), 16, 3), (4, 2, (500, 500), 16, 0),
                                                            (5, 3, (64, 48), 8, 0)])
def test_assemble_matches_the_layout_on_random_bytes(nranks, frames, size, tile, offset, gpu_available):
    """rt_assemble_tiles_device against a numpy restatement of the layout, on random shard bytes: the
    LDS-staged kernel (16x16 tiles, width a multiple of 16, whole gather, 16-B aligned buffers: partial
    tile chunks, partial bottom tile rows, 1-8 ranks) and the per-piece kernel (other widths, 8x8 tiles,
    an output 3 bytes off alignment) leave the same frames, and nothing outside them."""
    import torch
    w, h = size
    T = ((w + tile - 1) // tile) * ((h + tile - 1) // tile)
    slots = (frames * T + nranks - 1) // nranks
    rng = np.random.default_rng(nranks * 1000 + w)
    gathered = rng.integers(0, 256, nranks * slots * tile * tile * 3, dtype=np.uint8)
    d_g = torch.from_numpy(gathered).to("cuda:0")
    n = frames * h * w * 3
    d_out = torch.full((n + offset + 64,), 7, dtype=torch.uint8, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    R.assemble_tiles_device(0, w, h, tile, tile, frames, nranks, d_g.data_ptr(), d_g.numel(), d_out.data_ptr() + offset, n,
                            stream)
    got = d_out.cpu().numpy()
    assert np.array_equal(got[offset:offset + n].reshape(frames, h, w, 3), _unpermute_reference(gathered, w, h, tile, frames, nranks))
    assert (got[:offset] == 7).all() and (got[offset + n:] == 7).all()


@pytest.mark.parametrize("knobs", [{}, {"split_eighth": 4096}, {"quad_walk": 1, "steal_quarter": 4096}])
def test_strong_shares_settled_reassemble_to_the_frame(knobs, workdir, gpu_available):
    """bench.strong_shares' measurement: at N = 8 each rank's share of one C4 frame is
    rendered until its batch order and launch trials have settled (ordered launches: the split tiers,
    the trials' kernel and distribution), under the default and the wider split policies; the last
    render of every share, laid out as one gather lays them out and un-permuted, is the one-GPU frame
    byte for byte, and the shares' ray counts add up to the frame's."""
    import torch
    w, h, N = 1920, 1080, 8
    p = R.RenderParams(width=w, height=h, pf=1, max_lvl=3, lights=LIGHTS)
    T = (w // 16) * ((h + 15) // 16)
    shard = ((T + N - 1) // N) * 16 * 16 * 3
    stream = torch.cuda.current_stream().cuda_stream
    with R.Scene.load(scene_path("syn:C4", workdir), device=0) as sc:
        for k, v in knobs.items():
            sc.tune(k, v)
        full, c1 = _frame(sc, p)
        gathered = torch.full((N * shard,), 7, dtype=torch.uint8, device="cuda:0")
        total = np.zeros(3, np.uint64)
        for r in range(N):
            part = gathered[r * shard:(r + 1) * shard]
            sc.render_tiles_device(p, 16, 16, r, N, part.data_ptr(), part.numel(), stream)   # (resets the trials)
            torch.cuda.synchronize()
            n = 1
            while n < 64 and sc.trials()["choice"] < 0:
                sc.render_tiles_device(p, 16, 16, r, N, part.data_ptr(), part.numel(), stream)
                torch.cuda.synchronize()
                n += 1
            for _ in range(4):
                sc.render_tiles_device(p, 16, 16, r, N, part.data_ptr(), part.numel(), stream)
            _, c = sc.render_tiles_device(p, 16, 16, r, N, part.data_ptr(), part.numel(), stream, want_counts=True)
            total += c
            assert sc.trials()["choice"] >= 0, (r, n)
        out = torch.zeros(h * w * 3, dtype=torch.uint8, device="cuda:0")
        R.assemble_tiles_device(0, w, h, 16, 16, 1, N, gathered.data_ptr(), gathered.numel(), out.data_ptr(), out.numel(), stream)
        got = out.view(h, w, 3).cpu().numpy()
    assert np.array_equal(got, full)
    assert [int(x) for x in total] == [int(x) for x in c1]


def test_render_frames_sharded_world1(workdir, gpu_available):
    import torch
    comm = R.Comm(0, 0, 1, R.Comm.unique_id())
    assert comm.info() == (0, 1, 0)
    p = R.RenderParams(width=320, height=180, pf=2, max_lvl=3, lights=LIGHTS)
    with R.Scene.load(scene_path("syn:C4", workdir), device=0) as sc:
        full, c1 = _frame(sc, p)
        for frames in (1, 2):
            out = torch.zeros(frames * 180 * 320 * 3, dtype=torch.uint8, device="cuda:0")
            c = sc.render_frames_sharded(p, comm, 16, 16, frames, out.data_ptr(), out.numel(),
                                         torch.cuda.current_stream().cuda_stream, want_counts=True)
            got = out.view(frames, 180, 320, 3).cpu().numpy()
            for f in range(frames):
                assert np.array_equal(got[f], full)
            assert [int(x) for x in c] == [frames * int(x) for x in c1]
        with pytest.raises(R.RtError):   # rank 0 must pass an output buffer
            sc.render_frames_sharded(p, comm, 16, 16, 1, None, 0)
    comm.check()
    comm.close()


def test_render_frames_sharded_pipelined_world1(workdir, gpu_available):
    """rt_comm_set_pipeline 2: each call renders on the communicator's render
    stream into one of two alternating shards while the previous call gathers and un-permutes on the
    exchange stream (and, with the scene's frames in flight, beside the previous call's render).
    Twelve back-to-back calls (one and two frames each) into three rotating output
    buffers, with no host synchronisation between them: every output equals the one-GPU frame once
    the caller's stream has passed it; a counted call in the middle drains the pipeline; depth 1
    again afterwards."""
    import torch
    comm = R.Comm(0, 0, 1, R.Comm.unique_id())
    p = R.RenderParams(width=320, height=180, pf=2, max_lvl=3, lights=LIGHTS)
    st = torch.cuda.current_stream()
    with R.Scene.load(scene_path("syn:C4", workdir), device=0) as sc:
        full, c1 = _frame(sc, p)
        comm.set_pipeline(2)
        for frames, fif in ((1, 1), (2, 1), (1, 2), (2, 2)):
            sc.tune("frames_in_flight", fif)   # (2: consecutive calls' renders overlap too)
            outs = [torch.full((frames * 180 * 320 * 3,), 7, dtype=torch.uint8, device="cuda:0") for _ in range(3)]
            for i in range(12):
                o = outs[i % 3]
                if i >= 3:   # written by call i - 3: check it before reusing it
                    st.synchronize()
                    got = o.view(frames, 180, 320, 3).cpu().numpy()
                    for f in range(frames):
                        assert np.array_equal(got[f], full), (frames, fif, i - 3, f)
                    o.fill_(7)
                if i == 6:   # a counted call drains the pipeline and runs in order
                    c = sc.render_frames_sharded(p, comm, 16, 16, frames, o.data_ptr(), o.numel(), st.cuda_stream,
                                                 want_counts=True)
                    assert [int(x) for x in c] == [frames * int(x) for x in c1]
                else:
                    sc.render_frames_sharded(p, comm, 16, 16, frames, o.data_ptr(), o.numel(), st.cuda_stream)
            st.synchronize()
            for o in outs:
                got = o.view(frames, 180, 320, 3).cpu().numpy()
                for f in range(frames):
                    assert np.array_equal(got[f], full), (frames, fif)
        sc.tune("frames_in_flight", 1)
        comm.set_pipeline(1)
        out = torch.zeros(180 * 320 * 3, dtype=torch.uint8, device="cuda:0")
        sc.render_frames_sharded(p, comm, 16, 16, 1, out.data_ptr(), out.numel(), st.cuda_stream)
        assert np.array_equal(out.view(180, 320, 3).cpu().numpy(), full)
        with pytest.raises(R.RtError):
            comm.set_pipeline(3)
    comm.check()
    comm.close()


WORKER = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[5], sys.argv[5] + "/tests"]
import raytracert_amd as R
from _util import scene_path
rank, n, uid_file, out_file = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
torch.cuda.set_device(rank)
comm = R.Comm(rank, rank, n, open(uid_file, "rb").read())
sc = R.Scene.load(scene_path("syn:F3", "/tmp/rt_sharded_%d" % rank), device=rank)
p = R.RenderParams(width=100, height=70, pf=2, max_lvl=3, lights=[(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)])
out = torch.zeros(2 * 70 * 100 * 3, dtype=torch.uint8, device="cuda:%d" % rank)
c = sc.render_frames_sharded(p, comm, 16, 16, 2, out.data_ptr() if rank == 0 else None, out.numel() if rank == 0 else 0,
                             torch.cuda.current_stream().cuda_stream, want_counts=True)
if rank == 0:
    np.save(out_file, out.cpu().numpy())
comm.close()
"""


def test_render_frames_sharded_two_processes(workdir, tmp_path, gpu_available):
    if gpu_available < 2:
        pytest.skip("one GPU visible: RCCL refuses two ranks on one device (covered by the composition test)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    uid = tmp_path / "uid"
    uid.write_bytes(R.Comm.unique_id())
    script = tmp_path / "worker.py"
    script.write_text(WORKER)
    out = str(tmp_path / "frames.npy")
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, str(script), str(r), "2", str(uid), out, root], env=env) for r in range(2)]
    assert [p.wait(timeout=180) for p in procs] == [0, 0]
    p = R.RenderParams(width=100, height=70, pf=2, max_lvl=3, lights=LIGHTS)
    with R.Scene.load(scene_path("syn:F3", workdir), device=0) as sc:
        full, _ = _frame(sc, p)
    got = np.load(out).reshape(2, 70, 100, 3)
    assert np.array_equal(got[0], full) and np.array_equal(got[1], full)


def test_bench_multi_rank_rehearsal(tmp_path, gpu_available):
    """bench.py's N>1 step (interleaved tiles per rank, one gather to rank 0, the library's
    un-permute, max-over-ranks timing, the strong-scaling re-run) with two ranks sharing the one
    GPU over gloo (--rehearse): every assembled frame equals the one-GPU frame."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29533", os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--rehearse", "--workload", "c2", "--no-cpu", "--no-bf-roofline", "--no-cold",
           "--no-path-compare", "--frames-per-call", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 2 and d["config"]["frames_per_step"] == 2 and d["config"]["steps_per_call"] == 1
    assert d["rehearsal"]["frames_checked"] == 2 and d["rehearsal"]["all_equal_one_gpu_frame"]
    assert d["config"]["rays_per_step"] == 2 * 494405 and "strong" in d


def test_bench_multi_rank_rehearsal_steps_per_call(tmp_path, gpu_available):
    """The N>1 weak step with --frames-per-call 4: each rank renders its share of 4 steps' frames in one
    call, one gather, one un-permute of 8 frames; rays and frames are still reported per step."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29534", os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "8",
           "--warmup", "4", "--frames-per-call", "4", "--rehearse", "--workload", "c2", "--no-cpu", "--no-bf-roofline",
           "--no-cold", "--no-path-compare"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["config"]["frames_per_step"] == 2 and d["config"]["steps_per_call"] == 4
    assert d["rehearsal"]["frames_checked"] == 8 and d["rehearsal"]["all_equal_one_gpu_frame"]
    assert d["config"]["rays_per_step"] == 2 * 494405
