"""ctypes binding of the CPU restatement (oracle/build/librt_oracle.so).

TEST INFRASTRUCTURE ONLY: importable from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg. The product package (raytracert_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "librt_oracle.so")

MAX_LIGHTS = 16
ALL_FEATURES = 0x3F


class OraParams(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32),
        ("pfx", C.c_int32), ("pfy", C.c_int32),
        ("max_lvl", C.c_int32), ("flags", C.c_uint32),
        ("n_lights", C.c_int32), ("seed", C.c_int32),
        ("lights", (C.c_float * 3) * MAX_LIGHTS),
        ("camera_pos", C.c_float * 3),
        ("corners", (C.c_float * 3) * 8),
        ("light_list", C.c_void_p),   # n_lights x 3 floats (any count) or NULL
    ]


class OraMaterial(C.Structure):
    _fields_ = [
        ("Kd", C.c_float * 3), ("Ka", C.c_float * 3), ("Ks", C.c_float * 3),
        ("Ns", C.c_float), ("Ni", C.c_float), ("Tr", C.c_float),
        ("illum", C.c_int32), ("flags", C.c_uint32),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle library missing: {LIB_PATH} (run `make -C oracle`)")
        L = C.CDLL(LIB_PATH)
        L.ora_load_obj.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        L.ora_load_obj.restype = C.c_int
        L.ora_free.argtypes = [C.c_void_p]
        L.ora_counts.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.ora_export.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ora_ray_intersect_triangle.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.ora_ray_intersect_triangle.restype = C.c_int
        L.ora_ray_intersect_triangle_batch.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ora_intersect_mesh.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ora_intersect_mesh.restype = C.c_int
        L.ora_perform_ray_tracing.argtypes = [C.c_void_p, C.POINTER(OraParams), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.ora_render.argtypes = [C.c_void_p, C.POINTER(OraParams), C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                 C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        L.ora_default_corners.argtypes = [C.c_int32, C.c_int32, C.c_void_p]
        L.ora_debug_trace.argtypes = [C.c_void_p, C.POINTER(OraParams), C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
        L.ora_debug_trace.restype = C.c_int32
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def default_corners(width: int, height: int) -> np.ndarray:
    out = np.zeros((8, 3), np.float32)
    lib().ora_default_corners(width, height, _ptr(out))
    return out


STOCHASTIC = 1 << 8      # RT_STOCHASTIC: jittered sub-samples (include/raytracert.h)
DEFAULT_SEED = 0x5EED


class OraDebugBounce(C.Structure):
    _fields_ = [
        ("origin", C.c_float * 3), ("dest", C.c_float * 3), ("hit", C.c_float * 3),
        ("triangle", C.c_int32), ("level", C.c_int32), ("shadowed", C.c_uint32), ("lit", C.c_uint32),
    ]


def make_params(width, height, pf=1, max_lvl=0, lights=((0.0, 0.0, 4.0),), flags=ALL_FEATURES,
                camera_pos=(0.0, 0.0, 4.0), corners=None, seed=DEFAULT_SEED, pfy=None) -> OraParams:
    p = OraParams()
    p.width, p.height, p.pfx, p.pfy = width, height, pf, pf if pfy is None else pfy
    p.max_lvl, p.flags, p.n_lights = max_lvl, flags, len(lights)
    p.seed = seed
    for i, l in enumerate(lights[:MAX_LIGHTS]):
        for k in range(3):
            p.lights[i][k] = l[k]
    if len(lights) > MAX_LIGHTS:   # the reference's light list is unbounded: the rest through light_list
        arr = np.ascontiguousarray(np.asarray(lights, np.float32).reshape(len(lights), 3))
        p._light_list_keepalive = arr
        p.light_list = arr.ctypes.data
    for k in range(3):
        p.camera_pos[k] = camera_pos[k]
    cs = default_corners(width, height) if corners is None else np.asarray(corners, np.float32)
    for i in range(8):
        for k in range(3):
            p.corners[i][k] = float(cs[i, k])
    return p


class OracleScene:
    def __init__(self, path: str):
        h = C.c_void_p()
        rc = lib().ora_load_obj(path.encode(), C.byref(h))
        if rc != 0:
            raise OSError(f"oracle: cannot open {path}")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_free(self.h)
            self.h = None

    def counts(self):
        nv, nt, nm = C.c_int32(), C.c_int32(), C.c_int32()
        lib().ora_counts(self.h, C.byref(nv), C.byref(nt), C.byref(nm))
        return nv.value, nt.value, nm.value

    def export(self):
        nv, nt, nm = self.counts()
        verts = np.zeros((nv, 3), np.float32)
        tri = np.zeros((nt, 3), np.uint32)
        tmat = np.zeros(nt, np.uint32)
        mats = (OraMaterial * max(nm, 1))()
        normals = np.zeros((nt, 3), np.float32)
        lib().ora_export(self.h, _ptr(verts), _ptr(tri), _ptr(tmat), C.cast(mats, C.c_void_p), _ptr(normals))
        mat_list = []
        for i in range(nm):
            m = mats[i]
            mat_list.append(dict(Kd=tuple(m.Kd), Ka=tuple(m.Ka), Ks=tuple(m.Ks), Ns=m.Ns, Ni=m.Ni, Tr=m.Tr,
                                 illum=m.illum, flags=m.flags))
        return dict(vertices=verts, triangles=tri, tri_mat=tmat, materials=mat_list, normals=normals)

    def intersect_mesh(self, origin, dest):
        o = np.asarray(origin, np.float32)
        d = np.asarray(dest, np.float32)
        I = np.zeros(3, np.float32)
        idx = lib().ora_intersect_mesh(self.h, _ptr(o), _ptr(d), _ptr(I))
        return idx, I

    def trace(self, params: OraParams, origin, dest):
        o = np.asarray(origin, np.float32)
        d = np.asarray(dest, np.float32)
        rgb = np.zeros(3, np.float32)
        counts = np.zeros(3, np.uint64)
        lib().ora_perform_ray_tracing(self.h, C.byref(params), _ptr(o), _ptr(d), _ptr(rgb), _ptr(counts))
        return rgb, counts

    def debug_trace(self, params: OraParams, origin, dest, max_bounces=256):
        """Every trace() call of one ray's chain (ora_debug_trace): (bounces, rgb), bounces as
        dicts with the fields of rt_debug_bounce."""
        buf = (OraDebugBounce * max_bounces)()
        rgb = np.zeros(3, np.float32)
        o = np.ascontiguousarray(origin, np.float32).reshape(3)
        d = np.ascontiguousarray(dest, np.float32).reshape(3)
        n = lib().ora_debug_trace(self.h, C.byref(params), _ptr(o), _ptr(d), buf, max_bounces, _ptr(rgb))
        out = []
        for b in buf[: min(n, max_bounces)]:
            out.append(dict(origin=np.array(b.origin[:], np.float32), dest=np.array(b.dest[:], np.float32),
                            hit=np.array(b.hit[:], np.float32), triangle=b.triangle, level=b.level,
                            shadowed=b.shadowed, lit=b.lit))
        return out, rgb

    def render(self, params: OraParams, x0=0, y0=0, w=None, h=None, nthreads=None):
        w = params.width if w is None else w
        h = params.height if h is None else h
        nthreads = nthreads or min(8, os.cpu_count() or 1)
        f32 = np.zeros((h, w, 3), np.float32)
        u8 = np.zeros((h, w, 3), np.uint8)
        counts = np.zeros(3, np.uint64)
        lib().ora_render(self.h, C.byref(params), x0, y0, w, h, _ptr(f32), _ptr(u8), nthreads, _ptr(counts))
        return f32, u8, counts


def ray_intersect_triangle(R, T):
    R = np.ascontiguousarray(R, np.float32).reshape(6)
    T = np.ascontiguousarray(T, np.float32).reshape(9)
    I = np.zeros(3, np.float32)
    hit = lib().ora_ray_intersect_triangle(_ptr(R), _ptr(T), _ptr(I))
    return bool(hit), I


def ray_intersect_triangle_batch(R, T):
    """R: [n, 2, 3] (origin, dest) rays against one triangle T [3, 3] -> (hit[n] bool, I[n, 3])."""
    R = np.ascontiguousarray(R, np.float32).reshape(-1, 6)
    T = np.ascontiguousarray(T, np.float32).reshape(9)
    n = len(R)
    hit = np.zeros(n, np.uint8)
    I = np.zeros((n, 3), np.float32)
    lib().ora_ray_intersect_triangle_batch(_ptr(R), n, _ptr(T), _ptr(hit), _ptr(I))
    return hit.astype(bool), I
