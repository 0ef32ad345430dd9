#!/usr/bin/env python3
"""Where the drop-in's first frame trace loses ~8 ms (r05): rt_trace_frame_samples of the reference's
default frame (500x500, pf 3, max_lvl 10, RT_SAMPLES_RAY_RGB) into pinned buffers from rt_host_alloc,
timed on the host: buffer A twice, then a fresh buffer B twice, then A again; with rt_scene_reserve
first, as the drop-in's init() does. A slow first call into each fresh buffer means the cost is the
buffer's first DMA; a slow first call only means a one-time cost elsewhere.
Usage: python tools/first_trace_probe.py
"""
import ctypes as C
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402
import raytracert_amd as R  # noqa: E402
from raytracert_amd import _capi  # noqa: E402

wl = bench.WORKLOADS["ref_default"]
path = bench.workload_scene(wl["scene"], tempfile.mkdtemp())
p = R.RenderParams(width=wl["width"], height=wl["height"], pf=wl["pf"], max_lvl=wl["max_lvl"],
                   lights=[list(x) for x in wl["lights"]])
cp = p.to_c()
n = wl["width"] * wl["height"] * wl["pf"] ** 2
nbytes = 9 * 4 * n
lib = _capi.lib()


def alloc():
    ptr = C.c_void_p()
    _capi.check(lib.rt_host_alloc(nbytes, C.byref(ptr)))
    return ptr


with R.Scene.load(path, device=0) as sc:
    t0 = time.perf_counter()
    sc.reserve(p, 16, 16, _capi.SAMPLES_RAY_RGB)
    print(f"reserve {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
    A = alloc()
    B = alloc()
    for name, buf in (("A", A), ("A", A), ("B", B), ("B", B), ("A", A)):
        t0 = time.perf_counter()
        _capi.check(lib.rt_trace_frame_samples(sc._h, C.byref(cp), _capi.SAMPLES_RAY_RGB, buf, nbytes, None))
        print(f"trace into {name}: {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
    lib.rt_host_free(A)
    lib.rt_host_free(B)
