#!/usr/bin/env python3
"""rt_render_frames_sharded at pipeline depth 1 vs 2 (and 2 with the scene's frames in flight) on a world-1 RCCL communicator: per-call wall
time over K back-to-back calls (three rotating output buffers), for a bench workload. At N = 1 the
gather is a local copy; the un-permute is the real kernel. Usage: tools/sharded_pipeline.py [workload] [K]"""
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import torch  # noqa: E402

import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    wl = bench.WORKLOADS[name]
    path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
    p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"], lights=wl["lights"])
    comm = R.Comm(0, 0, 1, R.Comm.unique_id())
    st = torch.cuda.current_stream()
    nbytes = wl["width"] * wl["height"] * 3
    outs = [torch.zeros(nbytes, dtype=torch.uint8, device="cuda:0") for _ in range(3)]
    res = {"workload": name, "calls": K}
    with R.Scene.load(path, device=0) as sc:
        for depth, fif in ((1, 1), (2, 1), (2, 2), (1, 1), (2, 1), (2, 2)):
            comm.set_pipeline(depth)
            sc.tune("frames_in_flight", fif)
            for i in range(20):   # warm: batch order, launch trials
                sc.render_frames_sharded(p, comm, 16, 16, 1, outs[i % 3].data_ptr(), nbytes, st.cuda_stream)
                st.synchronize()
            t0 = time.perf_counter()
            for i in range(K):
                sc.render_frames_sharded(p, comm, 16, 16, 1, outs[i % 3].data_ptr(), nbytes, st.cuda_stream)
            st.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / K
            res.setdefault(f"depth{depth}_fif{fif}_ms_per_call", []).append(round(ms, 4))
        ref = torch.zeros(nbytes, dtype=torch.uint8, device="cuda:0")
        sc.render_frame_device(p.to_c(), 16, 16, ref.data_ptr(), nbytes, st.cuda_stream)
        st.synchronize()
        res["outputs_equal_frame"] = all(bool(torch.equal(o, ref)) for o in outs)
    comm.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
