"""Dead-lane shadow helpers (r05, rt_kernels.hip k_chain `dyn`): in a whole wave of the fused chain
launch, the lanes whose chain has ended (or that have no sample) pair with live lanes at every step and
walk every other light's shadow ray of their owner's hit. Only which lane walks a shadow ray changes, so
the frame must equal the frame with the helpers off (RT_TUNE_SHADOW_HELPERS 0) byte for byte, with the
same ray counts, for 2, 3 (an odd light for the unpaired owner's second walk), 4 and 8 lights, any-hit
and closest-hit shadows (F4 has a transparent material), ragged frames (lanes without a sample from the
start), and one tile against the oracle.
"""
import numpy as np
import pytest

import oracle as O
import raytracert_amd as R
from _util import scene_path

pytestmark = pytest.mark.gpu

LIGHTS = [(0.0, 0.0, 4.0), (1.5, 1.5, 4.0), (-1.2, 0.4, 3.0), (0.6, -1.4, 3.5), (2.0, -1.0, 3.5), (-2.0, -1.0, 3.5),
          (0.3, 2.2, 2.0), (0.0, 0.0, 1.0)]


def _frame(sc, p):
    import torch
    fb = torch.zeros(p.height * p.width * 3, dtype=torch.uint8, device="cuda:0")
    c = sc.render_frame_device(p, 16, 16, fb.data_ptr(), fb.numel(), torch.cuda.current_stream().cuda_stream,
                               want_counts=True)
    torch.cuda.synchronize()
    return fb.view(p.height, p.width, 3).cpu().numpy(), [int(x) for x in c]


@pytest.mark.parametrize("n_lights", [2, 3, 4, 8])
@pytest.mark.parametrize("spec,w,h,pf,max_lvl", [("syn:F3", 131, 77, 1, 3), ("syn:F4", 96, 54, 2, 4),
                                                 ("ref:dodgeColorTest.obj", 170, 120, 1, 3)])
def test_dead_lane_helpers_keep_the_frame(spec, w, h, pf, max_lvl, n_lights, workdir, gpu_available):
    path = scene_path(spec, workdir)
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=max_lvl, lights=LIGHTS[:n_lights])
    frames = {}
    for helpers in (1, 0):
        with R.Scene.load(path, device=0) as sc:
            sc.tune("shadow_helpers", helpers)
            for k in range(3):   # cold, then ordered launches (the pairing does not depend on the order)
                frames[(helpers, k)] = _frame(sc, p)
    ref_img, ref_counts = frames[(0, 2)]
    for key, (img, counts) in frames.items():
        assert np.array_equal(img, ref_img), key
        assert counts == ref_counts, key
    x0, y0 = (w // 2) & ~15, (h // 2) & ~15
    tw, th = min(16, w - x0), min(16, h - y0)
    op = O.make_params(w, h, pf, max_lvl, lights=LIGHTS[:n_lights])
    _, ou8, _ = O.OracleScene(path).render(op, x0, y0, tw, th, nthreads=16)
    assert np.array_equal(ref_img[y0:y0 + th, x0:x0 + tw], ou8)
