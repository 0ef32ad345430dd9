"""raytracert_amd — MI355X-native (gfx950) drop-in for the render path of wmorssink/raytracert.

The product is librtamd.so (C-ABI in include/raytracert.h): OBJ/MTL loading with the
reference's semantics, and hand-written HIP kernels for the per-pixel primary ray, the recursive
shadow/reflection/refraction trace and the brute-force closest-hit over Mesh::triangles. This
package is a thin Python mirror of that interface for tests, the benchmark and multi-GPU
orchestration (torch.distributed over RCCL).
"""
from ._capi import ALL_FEATURES, RtError, RT_HOST_ONLY  # noqa: F401
from .api import (Comm, RenderParams, Scene, assemble_tiles_device, default_corners, device_count,  # noqa: F401
                  load_mtl, ray_intersect_triangle, write_ppm, PpmWriter)

__all__ = ["Scene", "RenderParams", "Comm", "assemble_tiles_device", "default_corners", "write_ppm", "PpmWriter", "device_count", "ray_intersect_triangle", "load_mtl", "RtError",
           "ALL_FEATURES", "RT_HOST_ONLY"]
