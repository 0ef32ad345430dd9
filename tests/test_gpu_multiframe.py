"""rt_render_frames_device: several views of one frame geometry in one chain launch (VERDICT r04
"What's weak" 5 / "Next round" 6: frames that overlap without a second stream, so without depending
on two streams landing on different hardware queues).

The launch's wave tasks cycle over the frames (task t is frame t % K's task t / K), each frame reading
its own corner rays and writing its own buffer. Every frame must equal that view rendered alone, byte
for byte, and the counts the sum of the single-view counts; calls that cannot be one launch (two render
pipelines, more than 16 lights, the quad tier) render the frames one after another with the same
bytes; frames that differ in anything but their corners are refused.
"""
import numpy as np
import pytest

import oracle as O
import raytracert_amd as R
from _util import scene_path
from raytracert_amd import scenes

pytestmark = pytest.mark.gpu

C4 = dict(spec="syn:C4", w=1920, h=1080, pf=1, max_lvl=3, lights=[(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)])
REF = dict(spec="ref:dodgeColorTest.obj", w=500, h=500, pf=3, max_lvl=10, lights=[(0.0, 0.0, 4.0)])


def _views(wl, k, step=3.0):
    return [R.RenderParams(width=wl["w"], height=wl["h"], pf=wl["pf"], max_lvl=wl["max_lvl"], lights=wl["lights"],
                           corners=scenes.orbit_corners(wl["w"], wl["h"], i, step)) for i in range(k)]


def _single(sc, torch, dev, p):
    buf = torch.zeros(p.height * p.width * 3, dtype=torch.uint8, device=dev)
    c = sc.render_frame_device(p, 16, 16, buf.data_ptr(), buf.numel(), torch.cuda.current_stream(dev).cuda_stream,
                               want_counts=True)
    return buf, c


@pytest.mark.parametrize("name,knobs", [("c4", {}), ("c4", {"chain_split": 4}), ("ref_default", {}),
                                        ("c4", {"pipes": 2}), ("c4", {"quad_walk": 1, "steal_quarter": 64})])
def test_frames_in_one_launch_equal_single_frames(name, knobs, workdir, gpu_available):
    import torch
    wl = C4 if name == "c4" else REF
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    views = _views(wl, 8)
    with R.Scene.load(scene_path(wl["spec"], workdir), device=0) as sc:
        for k, v in knobs.items():
            sc.tune(k, v)
        singles = [_single(sc, torch, dev, p) for p in views]
        torch.cuda.synchronize(dev)
        for it in range(12):   # cold, re-sorted and (after the trials) ordered launches; K = 2, 3, 4, 8
            K = (2, 3, 4, 8)[it % 4]
            bufs = [torch.full((wl["h"] * wl["w"] * 3,), 7, dtype=torch.uint8, device=dev) for _ in range(K)]
            counts = sc.render_frames_device(views[:K], 16, 16, [b.data_ptr() for b in bufs], bufs[0].numel(), st.cuda_stream,
                                             want_counts=(it % 3 == 0))
            torch.cuda.synchronize(dev)
            for f in range(K):
                assert torch.equal(bufs[f], singles[f][0]), (it, K, f)
            if counts is not None:
                assert [int(x) for x in counts] == [sum(int(singles[f][1][k]) for f in range(K)) for k in range(3)]
        # the views are distinct, and one of them matches the oracle on a tile of its sphere region
        assert len({s[0].cpu().numpy().tobytes().__hash__() for s in singles}) == 8
        x0, y0 = (wl["w"] // 2) & ~15, (wl["h"] // 2) & ~15
        img = singles[3][0].cpu().numpy().reshape(wl["h"], wl["w"], 3)
        op = O.make_params(wl["w"], wl["h"], wl["pf"], wl["max_lvl"], lights=wl["lights"], corners=views[3].corners)
        _, ou8, _ = O.OracleScene(scene_path(wl["spec"], workdir)).render(op, x0, y0, 16, 16, nthreads=16)
        assert np.array_equal(img[y0:y0 + 16, x0:x0 + 16], ou8)


def test_multiframe_workspace_grows_by_the_deep_records_only(workdir, gpu_available):
    """eight views at the reference's defaults (max_lvl 10: chain records past the three
    LDS steps) in one launch keep each frame's deep records at sample + frame x samples in chain_local;
    only that array grows with the frames (7 more frames x 2.36M samples x 11 steps x 16 B), not the
    whole ~1 GB per-frame workspace (~8.5 GB before), and the call renders in one launch (no fallback)."""
    import torch
    dev = torch.device("cuda", 0)
    views = _views(REF, 8)
    # (the workspace's samples: whole 16 x 16 tiles, the frame's edge tiles padded)
    cap, steps = ((REF["w"] + 15) // 16) * ((REF["h"] + 15) // 16) * 256 * REF["pf"] ** 2, REF["max_lvl"] + 1
    with R.Scene.load(scene_path(REF["spec"], workdir), device=0) as sc:
        one, _ = _single(sc, torch, dev, views[7])
        torch.cuda.synchronize(dev)
        b1, f1 = sc.workspace_bytes()
        bufs = [torch.zeros(REF["h"] * REF["w"] * 3, dtype=torch.uint8, device=dev) for _ in range(8)]
        sc.render_frames_device(views, 16, 16, [b.data_ptr() for b in bufs], bufs[0].numel(),
                                torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        b8, f8 = sc.workspace_bytes()
        assert f1 == f8 == 0
        assert b1 < b8 <= b1 + 7 * cap * steps * 16 + 4096, (b1, b8)
        assert b8 < 4 * b1
        assert torch.equal(bufs[7], one)


def test_frames_in_one_launch_two_in_flight(workdir, gpu_available):
    """Two-frame calls on two streams with RT_TUNE_FRAMES_IN_FLIGHT 2 (each call on its own pipeline)."""
    import torch
    dev = torch.device("cuda", 0)
    views = _views(C4, 4)
    with R.Scene.load(scene_path(C4["spec"], workdir), device=0) as sc:
        singles = [_single(sc, torch, dev, p)[0] for p in views]
        sc.tune("frames_in_flight", 2)
        streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
        bufs = [torch.zeros(C4["h"] * C4["w"] * 3, dtype=torch.uint8, device=dev) for _ in range(4)]
        for it in range(10):
            pair = (0, 1) if it % 2 == 0 else (2, 3)
            sc.render_frames_device([views[i] for i in pair], 16, 16, [bufs[i].data_ptr() for i in pair], bufs[0].numel(),
                                    streams[it % 2].cuda_stream)
            if it % 2 == 1:
                torch.cuda.synchronize(dev)
                for i in range(4):
                    assert torch.equal(bufs[i], singles[i]), (it, i)


def test_frames_differing_beyond_corners_are_refused(workdir, gpu_available):
    import torch
    dev = torch.device("cuda", 0)
    views = _views(C4, 2)
    views[1].lights = [(0.0, 0.0, 4.0)]
    with R.Scene.load(scene_path(C4["spec"], workdir), device=0) as sc:
        bufs = [torch.zeros(C4["h"] * C4["w"] * 3, dtype=torch.uint8, device=dev) for _ in range(2)]
        with pytest.raises(R.RtError):
            sc.render_frames_device(views, 16, 16, [b.data_ptr() for b in bufs], bufs[0].numel())
