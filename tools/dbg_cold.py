"""Debug: ray counts of cold (estimate-ordered) and warm renders against screen order, alternating
the rect entry (scene stream) and the device-frame entry (torch stream) as the parity test does."""
import os, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch
import raytracert_amd as R
from _util import scene_path
d = tempfile.mkdtemp()
w, h = 320, 180
p = R.RenderParams(width=w, height=h, pf=1, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
for mode in ("alt", "alt_sync", "rect_only"):
    with R.Scene.load(scene_path("syn:C4", d), device=0) as sc:
        sc.tune("batch_order", 0)
        ref, _, refc = sc.render(p)
        fb0 = torch.zeros(h * w * 3, dtype=torch.uint8, device="cuda:0")
        sc.render_frame_device(p, 16, 16, fb0.data_ptr(), fb0.numel(), torch.cuda.current_stream().cuda_stream)
        sc.tune("batch_order", 1)
        for est in (1, 0, 1):
            sc.tune("cold_estimate", est)
            sc.tune("forget_order", 1)
            for k in range(3):
                u8, _, c = sc.render(p)
                ok = [int(x) for x in c] == [int(x) for x in refc] and np.array_equal(u8, ref)
                fbok = None
                if mode != "rect_only":
                    fb = torch.full((h * w * 3,), 7, dtype=torch.uint8, device="cuda:0")
                    sc.render_frame_device(p, 16, 16, fb.data_ptr(), fb.numel(), torch.cuda.current_stream().cuda_stream)
                    if mode == "alt_sync":
                        torch.cuda.synchronize()
                    fbok = bool(torch.equal(fb, fb0))
                print(mode, "est", est, "render", k, "ok", ok, [int(x) for x in c], "fb_ok", fbok, flush=True)
