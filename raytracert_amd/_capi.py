"""ctypes binding of librtamd.so (include/raytracert.h).

The library is built in-tree (raytracert_amd/librtamd.so, `make -C raytracert_amd`). There is
no fallback: if the shared object is missing or fails to load, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# RTAMD_LIB selects another in-tree build of the same library (A/B of kernel variants, tools/)
LIB_PATH = os.environ.get("RTAMD_LIB") or os.path.join(HERE, "librtamd.so")
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "raytracert.h")
TUNE_HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "raytracert_tune.h")   # tuning + diagnostics

RT_OK = 0
RT_E_IO = -1
RT_E_PARSE = -2
RT_E_HIP = -3
RT_E_ARG = -4
RT_E_NOMEM = -5
RT_E_NODEV = -6
RT_E_RCCL = -7
COMM_ID_BYTES = 128
RT_HOST_ONLY = -1
RT_MAX_LIGHTS = 16        # lights held inline in rt_params; more through rt_params.light_list
RT_LIGHTS_LIMIT = 65536
RT_TRIAL_INFO_FIELDS, RT_MAX_TRIALS = 7, 10
SAMPLES_RGB, SAMPLES_RAY_RGB = 3, 9   # rt_trace_frame_samples record layouts
RT_WS_ARRAYS = 22   # rt_workspace_layout arrays

AMBIENT, DIFFUSE, SPECULAR, REFLECTION, SHADOWS, REFRACTION = (1 << i for i in range(6))
ALL_FEATURES = 0x3F

HAS_KD, HAS_KA, HAS_KS, HAS_NS, HAS_NI, HAS_TR, HAS_ILLUM = (1 << i for i in range(7))

KERNEL_CLOSEST_HIT, KERNEL_SHADOW, KERNEL_SHADE, KERNEL_FRAME, KERNEL_CHAIN = range(5)
KERNEL_KINDS = 5
ACCEL_BRUTE_FORCE, ACCEL_BVH = 0, 1
TUNE_XCD_SPLIT, TUNE_BVH_GRID, TUNE_BVH_WIDTH, TUNE_LDS_STACK, TUNE_PIPES, TUNE_SHADOW_VIRTUAL = 0, 1, 2, 3, 4, 5
TUNE_PIPE_BATCHES, TUNE_PIPE_PRIORITY, TUNE_WAVE_TRAVERSAL, TUNE_CHAIN_FROM = 6, 7, 8, 9
TUNE_CHAIN_SPLIT, TUNE_TOP_NODES, TUNE_BATCH_ORDER, TUNE_ORDER_EVERY, TUNE_FUSE_PIXELS = 12, 13, 15, 17, 18
TUNE_CHAIN_REFILL, TUNE_REFILL_GRID, TUNE_WAVE_STEAL = 19, 20, 21
TUNE_COLD_ESTIMATE, TUNE_FORGET_ORDER = 24, 25
TUNE_STEAL_HALF, TUNE_STEAL_QUARTER = 22, 23
TUNE_SPLIT_EIGHTH, TUNE_PRIORITY_BATCHES, TUNE_PIXEL_ORDER, TUNE_DYN_GROUP = 26, 27, 28, 29
TUNE_SHADOW_HELPERS = 30
TUNE_FRAMES_IN_FLIGHT = 31
TUNE_ADOPT_ORDER = 32
TUNE_INFLIGHT_DYNAMIC = 33
TUNE_INFLIGHT_STREAMS = 34
TUNE_QUAD_WALK = 35
TUNE_MOTION_ORDER = 36
TUNE_ORDER_EARLY = 37
MAX_FRAMES_PER_CALL = 8   # RT_MAX_FRAMES_PER_CALL
BVH_INFO_FIELDS = 7
STOCHASTIC = 1 << 8
DEFAULT_SEED = 0x5EED
LOAD_PARALLEL, LOAD_SEQUENTIAL = 0, 1
LOAD_TEXCOORDS = 0x10
WORK_FIELDS = 6


class RtParams(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32),
        ("pfx", C.c_int32), ("pfy", C.c_int32),
        ("max_lvl", C.c_int32), ("flags", C.c_uint32),
        ("n_lights", C.c_int32), ("seed", C.c_int32),
        ("lights", (C.c_float * 3) * RT_MAX_LIGHTS),
        ("camera_pos", C.c_float * 3),
        ("corners", (C.c_float * 3) * 8),
        ("light_list", C.c_void_p),   # n_lights x 3 floats (any count) or NULL: lights[0..n_lights)
    ]


class RtDebugBounce(C.Structure):
    _fields_ = [
        ("origin", C.c_float * 3), ("dest", C.c_float * 3), ("hit", C.c_float * 3),
        ("triangle", C.c_int32), ("level", C.c_int32), ("shadowed", C.c_uint32), ("lit", C.c_uint32),
    ]


class RtMaterial(C.Structure):
    _fields_ = [
        ("Kd", C.c_float * 3), ("Ka", C.c_float * 3), ("Ks", C.c_float * 3),
        ("Ns", C.c_float), ("Ni", C.c_float), ("Tr", C.c_float),
        ("illum", C.c_int32), ("flags", C.c_uint32),
    ]


class RtError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"rt error {code}: {message}")
        self.code = code


_VP = C.c_void_p
_SIGNATURES = {
    "rt_last_error_string": ([], C.c_char_p),
    "rt_device_count": ([C.POINTER(C.c_int32)], C.c_int),
    "rt_scene_load_obj": ([C.c_char_p, C.c_int32, C.POINTER(_VP)], C.c_int),
    "rt_scene_load_obj_ex": ([C.c_char_p, C.c_int32, C.c_int32, C.POINTER(_VP)], C.c_int),
    "rt_scene_create": ([_VP, C.c_int32, _VP, _VP, C.c_int32, _VP, C.c_int32, C.c_int32, C.POINTER(_VP)], C.c_int),
    "rt_scene_destroy": ([_VP], None),
    "rt_scene_info": ([_VP, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)], C.c_int),
    "rt_scene_export": ([_VP, _VP, _VP, _VP, _VP, _VP], C.c_int),
    "rt_get_material": ([_VP, C.c_int32, C.POINTER(RtMaterial)], C.c_int),
    "rt_ray_intersect_triangle": ([C.c_int32, _VP, _VP, C.c_int32, _VP, _VP], C.c_int),
    "rt_intersect_mesh": ([_VP, _VP, _VP, C.c_int32, _VP, _VP], C.c_int),
    "rt_trace_rays": ([_VP, C.POINTER(RtParams), _VP, _VP, C.c_int32, _VP, _VP], C.c_int),
    "rt_debug_trace": ([_VP, C.POINTER(RtParams), _VP, _VP, _VP, C.c_int32, C.POINTER(C.c_int32), _VP], C.c_int),
    "rt_render_tile": ([_VP, C.POINTER(RtParams), C.c_int32, C.c_int32, C.c_int32, C.c_int32, _VP, _VP, _VP], C.c_int),
    "rt_trace_frame_samples": ([_VP, C.POINTER(RtParams), C.c_int32, _VP, C.c_size_t, _VP], C.c_int),
    "rt_host_alloc": ([C.c_size_t, C.POINTER(_VP)], C.c_int),
    "rt_scene_reserve": ([_VP, C.POINTER(RtParams), C.c_int32, C.c_int32, C.c_int32], C.c_int),
    "rt_render_frames_device": ([_VP, C.POINTER(RtParams), C.c_int32, C.c_int32, C.c_int32, C.POINTER(_VP), C.c_size_t, _VP, _VP],
                                C.c_int),
    "rt_host_free": ([_VP], None),
    "rt_render_frame_device": ([_VP, C.POINTER(RtParams), C.c_int32, C.c_int32, _VP, C.c_size_t, _VP, _VP], C.c_int),
    "rt_render_tiles_device": ([_VP, C.POINTER(RtParams), C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _VP,
                                C.c_size_t, _VP, C.POINTER(C.c_int32), _VP], C.c_int),
    "rt_default_corners": ([C.c_int32, C.c_int32, _VP], C.c_int),
    "rt_write_ppm": ([C.c_char_p, C.c_int32, C.c_int32, _VP], C.c_int),
    "rt_ppm_writer_open": ([C.c_char_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(_VP)], C.c_int),
    "rt_ppm_writer_write": ([_VP, _VP], C.c_int),
    "rt_ppm_writer_close": ([_VP], None),
    "rt_set_profiling": ([_VP, C.c_int32], C.c_int),
    "rt_kernel_stats": ([_VP, C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_double), C.POINTER(C.c_double)], C.c_int),
    "rt_reset_stats": ([_VP], C.c_int),
    "rt_work_stats": ([_VP, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double)], C.c_int),
    "rt_scene_set_accel": ([_VP, C.c_int32], C.c_int),
    "rt_scene_get_accel": ([_VP, C.POINTER(C.c_int32)], C.c_int),
    "rt_scene_bvh_info": ([_VP, _VP], C.c_int),
    "rt_work_detail": ([_VP, C.c_int32, _VP], C.c_int),
    "rt_diag_read": ([_VP, C.c_int64, C.c_int64, _VP], C.c_int),
    "rt_workspace_bytes": ([_VP, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)], C.c_int),
    "rt_workspace_layout": ([C.c_int64, C.c_int32, C.c_int32, C.POINTER(C.c_uint64), _VP], C.c_int),
    "rt_batch_durations": ([_VP, _VP, C.c_int64, C.POINTER(C.c_int64)], C.c_int),
    "rt_scene_trials": ([_VP, _VP, _VP], C.c_int),
    "rt_scene_bvh_digest": ([_VP, C.POINTER(C.c_uint64)], C.c_int),
    "rt_scene_bvh_validate": ([_VP], C.c_int),
    "rt_bvh_acceptance_box": ([_VP, _VP, _VP], C.c_int),
    "rt_scene_tune": ([_VP, C.c_int32, C.c_int32], C.c_int),
    "rt_scene_texcoords": ([_VP, C.POINTER(C.c_int32), _VP, _VP], C.c_int),
    "rt_load_mtl": ([C.c_char_p, C.POINTER(C.c_int32), _VP, C.c_int32, C.c_char_p, C.c_size_t], C.c_int),
    "rt_comm_unique_id": ([_VP], C.c_int),
    "rt_comm_init": ([C.c_int32, C.c_int32, C.c_int32, _VP, C.POINTER(_VP)], C.c_int),
    "rt_comm_destroy": ([_VP], None),
    "rt_comm_info": ([_VP, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)], C.c_int),
    "rt_comm_check": ([_VP], C.c_int),
    "rt_comm_set_pipeline": ([_VP, C.c_int32], C.c_int),
    "rt_render_frames_sharded": ([_VP, C.POINTER(RtParams), _VP, C.c_int32, C.c_int32, C.c_int32, _VP, C.c_size_t, _VP,
                                  _VP], C.c_int),
    "rt_assemble_tiles_device": ([C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _VP,
                                  C.c_size_t, _VP, C.c_size_t, _VP], C.c_int),
}

_lib = None


def header_symbols(paths=(HEADER_PATH, TUNE_HEADER_PATH)) -> list[str]:
    """Function names declared in include/raytracert.h and include/raytracert_tune.h."""
    if isinstance(paths, str):
        paths = (paths,)
    text = "".join(open(p).read() for p in paths)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", text)))


def lib() -> C.CDLL:
    """Load librtamd.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C raytracert_amd` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
        # torch bundles its own libamdhip64.so.7 / libhsa-runtime64; if it is loaded after
        # librtamd.so (which resolves /opt/rocm's), the process holds two HIP runtimes and torch
        # finds no GPU. Loading torch first makes librtamd bind to the already-loaded runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        ab = "RTAMD_LIB" in os.environ   # an A/B build of an older revision may lack newer entries
        for name, (args, res) in _SIGNATURES.items():
            if ab and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != RT_OK:
        msg = lib().rt_last_error_string()
        raise RtError(rc, msg.decode() if msg else "")
