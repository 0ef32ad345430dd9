"""A moving view (VERDICT r04 "What's missing" 2): the reference renders a new view per 'r' press
after the trackball turned it (traqueboule.h:103-165, main.cpp:355-358). Views of an orbit
(scenes.orbit_corners: the default C4 view turned about the world y axis, MyCameraPosition fixed
as main.cpp:222 computes it once) are rendered back to back with two frames in flight, the batch
order and launch trials carried over from view to view (the order's signature is the frame
geometry, not the camera). Every view's buffer must equal a fresh one-in-flight render of that
view, and sampled tiles of it the oracle's.
"""
import numpy as np
import pytest

import oracle as O
import raytracert_amd as R
from _util import scene_path
from raytracert_amd import scenes

pytestmark = pytest.mark.gpu

W, H = 1920, 1080
LIGHTS = [(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)]
VIEWS = 12
STEP_DEG = 2.0
TILES = [(944, 528), (640, 304), (1264, 720)]


def _params(k):
    return R.RenderParams(width=W, height=H, pf=1, max_lvl=3, lights=LIGHTS,
                          corners=scenes.orbit_corners(W, H, k, STEP_DEG))


def test_orbit_views_in_flight_equal_one_in_flight_and_oracle(workdir, gpu_available):
    import torch
    path = scene_path("syn:C4", workdir)
    dev = torch.device("cuda", 0)
    main = torch.cuda.current_stream(dev)
    cps = [_params(k).to_c() for k in range(VIEWS)]
    with R.Scene.load(path, device=0) as sc:
        ref = torch.zeros(H * W * 3, dtype=torch.uint8, device=dev)
        for _ in range(60):   # view 0 until its batch order is measured and its trials decided
            sc.render_frame_device(cps[0], 16, 16, ref.data_ptr(), ref.numel(), main.cuda_stream)
            torch.cuda.synchronize(dev)
            if sc.trials()["choice"] >= 0:
                break
        assert sc.trials()["choice"] >= 0
        sc.tune("frames_in_flight", 2)
        streams = [main, torch.cuda.Stream(dev)]
        bufs = [torch.full((H * W * 3,), 7, dtype=torch.uint8, device=dev) for _ in range(VIEWS)]
        for k in range(VIEWS):   # a new view per frame, two in flight
            sc.render_frame_device(cps[k], 16, 16, bufs[k].data_ptr(), bufs[k].numel(), streams[k % 2].cuda_stream)
        torch.cuda.synchronize(dev)
        assert sc.trials()["choice"] >= 0   # (carried over: no view re-ran the trials)
        sc.tune("frames_in_flight", 1)
        orc = O.OracleScene(path)
        distinct = set()
        for k in range(VIEWS):
            sc.render_frame_device(cps[k], 16, 16, ref.data_ptr(), ref.numel(), main.cuda_stream)
            torch.cuda.synchronize(dev)
            assert torch.equal(bufs[k], ref), f"view {k}"
            img = ref.cpu().numpy().reshape(H, W, 3)
            distinct.add(img.tobytes().__hash__())
            if k % 4 == 3:   # sampled tiles of every fourth view against the oracle
                op = O.make_params(W, H, 1, 3, lights=LIGHTS, corners=scenes.orbit_corners(W, H, k, STEP_DEG))
                for x0, y0 in TILES:
                    _, ou8, _ = orc.render(op, x0, y0, 16, 16, nthreads=16)
                    assert np.array_equal(img[y0:y0 + 16, x0:x0 + 16], ou8), (k, x0, y0)
        assert len(distinct) == VIEWS   # every view is a different image
