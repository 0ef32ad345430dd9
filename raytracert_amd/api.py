"""Python mirror of the reference's render-path interface, over the C-ABI.

Reference names kept (CG_Project/raytracing.h): `init` -> Scene.load (raytracing.h:19),
`intersectMesh` -> Scene.intersect_mesh (raytracing.cpp:161), `performRayTracing` ->
Scene.perform_ray_tracing (raytracing.h:33), `getMaterial` -> Scene.get_material
(raytracing.h:27), the 'r' key -> Scene.render (main.cpp:340-411), `produceRay` corners ->
default_corners (main.cpp:300-325), `Image::writeImage` -> write_ppm (main.cpp:102-128).
Every call goes to librtamd.so; errors raise RtError with the library's message.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

from . import _capi
from ._capi import ALL_FEATURES, RT_HOST_ONLY, RtMaterial, RtParams, check, lib


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def default_corners(width: int, height: int) -> np.ndarray:
    """The 8 corner vectors produceRay yields for the default view (origin00, dest00, origin01,
    dest01, origin10, dest10, origin11, dest11)."""
    out = np.zeros((8, 3), np.float32)
    check(lib().rt_default_corners(width, height, _ptr(out)))
    return out


def write_ppm(path: str, rgb_u8: np.ndarray) -> None:
    rgb = np.ascontiguousarray(rgb_u8, np.uint8)
    h, w = rgb.shape[:2]
    check(lib().rt_write_ppm(path.encode(), w, h, _ptr(rgb)))


class PpmWriter:
    """rt_ppm_writer_*: result.ppm written after every frame (main.cpp:405), the file kept mapped and
    each frame's bytes copied in by `threads` threads; the file holds write_ppm's bytes."""

    def __init__(self, path: str, width: int, height: int, threads: int = 8):
        self._h = C.c_void_p()
        self.width, self.height = width, height
        check(lib().rt_ppm_writer_open(path.encode(), width, height, threads, C.byref(self._h)))

    def write_ptr(self, host_ptr: int) -> None:
        """The frame at a host address (e.g. a pinned torch tensor's data_ptr()), width*height*3 bytes."""
        check(lib().rt_ppm_writer_write(self._h, C.c_void_p(host_ptr)))

    def write(self, rgb_u8: np.ndarray) -> None:
        rgb = np.ascontiguousarray(rgb_u8, np.uint8)
        if rgb.size != self.width * self.height * 3:
            raise ValueError("frame size differs from the writer's")
        self.write_ptr(rgb.ctypes.data)

    def close(self) -> None:
        if self._h:
            lib().rt_ppm_writer_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


@dataclass
class RenderParams:
    """Everything the reference reads from globals during a render (raytracing.cpp:15-29,
    raytracing.h:9-16). Defaults are the reference's own: pixelfactor 3, max_lvl 10, every
    feature on, one light at the camera position (0,0,4)."""
    width: int = 500
    height: int = 500
    pf: int = 3
    max_lvl: int = 10
    lights: Sequence[Sequence[float]] = ((0.0, 0.0, 4.0),)
    flags: int = ALL_FEATURES
    camera_pos: Sequence[float] = (0.0, 0.0, 4.0)
    corners: np.ndarray | None = field(default=None, repr=False)
    seed: int = _capi.DEFAULT_SEED   # RT_STOCHASTIC jitter seed (flags | STOCHASTIC)
    pfy: int | None = None           # pixelfactorY when it differs from pixelfactorX (= pf)

    def to_c(self) -> RtParams:
        """The C struct. Up to RT_MAX_LIGHTS lights go inline; more go through light_list, a float32
        array kept alive on the returned struct (the reference's light list is unbounded)."""
        n = len(self.lights)
        if n > _capi.RT_LIGHTS_LIMIT:
            raise ValueError(f"at most {_capi.RT_LIGHTS_LIMIT} lights")
        p = RtParams()
        p.width, p.height, p.pfx, p.pfy = self.width, self.height, self.pf, self.pf if self.pfy is None else self.pfy
        p.max_lvl, p.flags, p.n_lights = self.max_lvl, self.flags, n
        p.seed = int(self.seed)
        for i, l in enumerate(self.lights[:_capi.RT_MAX_LIGHTS]):
            for k in range(3):
                p.lights[i][k] = float(l[k])
        if n > _capi.RT_MAX_LIGHTS:
            arr = np.ascontiguousarray(np.asarray(self.lights, np.float32).reshape(n, 3))
            p._light_list_keepalive = arr
            p.light_list = arr.ctypes.data
        for k in range(3):
            p.camera_pos[k] = float(self.camera_pos[k])
        cs = default_corners(self.width, self.height) if self.corners is None else np.asarray(self.corners, np.float32)
        for i in range(8):
            for k in range(3):
                p.corners[i][k] = float(cs[i, k])
        return p


class Scene:
    """A loaded mesh bound to one GPU (or host-only with device=-1)."""

    def __init__(self, handle: C.c_void_p, device: int):
        self._h = handle
        self.device = device

    # -- construction ------------------------------------------------------------------------
    @classmethod
    def load(cls, path: str, device: int = 0, sequential: bool = False, threads: int = 0,
             texcoords: bool = False) -> "Scene":
        """init(fileName): Mesh::loadMesh + loadMtl + calculateNormals. The default parser is
        parallel (threads=0: automatic); sequential=True runs the line-by-line restatement (same
        result); texcoords=True also keeps Mesh::texcoords / Triangle::t (Scene.texcoords())."""
        h = C.c_void_p()
        flags = _capi.LOAD_SEQUENTIAL if sequential else (_capi.LOAD_PARALLEL | (int(threads) << 8))
        if texcoords:
            flags |= _capi.LOAD_TEXCOORDS
        check(lib().rt_scene_load_obj_ex(path.encode(), device, flags, C.byref(h)))
        return cls(h, device)

    @classmethod
    def create(cls, vertices, triangles, tri_mat, materials: Sequence[dict], device: int = 0) -> "Scene":
        v = np.ascontiguousarray(vertices, np.float32).reshape(-1, 3)
        t = np.ascontiguousarray(triangles, np.uint32).reshape(-1, 3)
        m = np.ascontiguousarray(tri_mat, np.uint32).reshape(-1)
        mats = (RtMaterial * len(materials))()
        for i, d in enumerate(materials):
            for k in range(3):
                mats[i].Kd[k] = d.get("Kd", (0, 0, 0))[k]
                mats[i].Ka[k] = d.get("Ka", (0, 0, 0))[k]
                mats[i].Ks[k] = d.get("Ks", (0, 0, 0))[k]
            mats[i].Ns, mats[i].Ni, mats[i].Tr = d.get("Ns", 0.0), d.get("Ni", 0.0), d.get("Tr", 0.0)
            mats[i].illum, mats[i].flags = d.get("illum", 0), d.get("flags", 0)
        h = C.c_void_p()
        check(lib().rt_scene_create(_ptr(v), len(v), _ptr(t), _ptr(m), len(m), C.cast(mats, C.c_void_p),
                                    len(materials), device, C.byref(h)))
        return cls(h, device)

    def close(self) -> None:
        if self._h:
            lib().rt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    # -- inspection --------------------------------------------------------------------------
    def counts(self) -> tuple[int, int, int]:
        nv, nt, nm = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib().rt_scene_info(self._h, C.byref(nv), C.byref(nt), C.byref(nm)))
        return nv.value, nt.value, nm.value

    def export(self) -> dict:
        nv, nt, nm = self.counts()
        verts = np.zeros((nv, 3), np.float32)
        tri = np.zeros((nt, 3), np.uint32)
        tmat = np.zeros(nt, np.uint32)
        normals = np.zeros((nt, 3), np.float32)
        mats = (RtMaterial * max(nm, 1))()
        check(lib().rt_scene_export(self._h, _ptr(verts), _ptr(tri), _ptr(tmat), C.cast(mats, C.c_void_p), _ptr(normals)))
        mat_list = [dict(Kd=tuple(m.Kd), Ka=tuple(m.Ka), Ks=tuple(m.Ks), Ns=m.Ns, Ni=m.Ni, Tr=m.Tr,
                         illum=m.illum, flags=m.flags) for m in list(mats)[:nm]]
        return dict(vertices=verts, triangles=tri, tri_mat=tmat, materials=mat_list, normals=normals)

    def texcoords(self) -> tuple[np.ndarray, np.ndarray]:
        """rt_scene_texcoords (a scene loaded with texcoords=True): (texcoords[n, 3] float32 with z = 0,
        tri_t[nt, 3] uint32), Mesh::texcoords and each Triangle::t."""
        n = C.c_int32()
        check(lib().rt_scene_texcoords(self._h, C.byref(n), None, None))
        tc = np.zeros((n.value, 3), np.float32)
        tt = np.zeros((self.counts()[1], 3), np.uint32)
        check(lib().rt_scene_texcoords(self._h, C.byref(n), _ptr(tc), _ptr(tt)))
        return tc, tt

    def get_material(self, triangle_index: int) -> dict:
        m = RtMaterial()
        check(lib().rt_get_material(self._h, triangle_index, C.byref(m)))
        return dict(Kd=tuple(m.Kd), Ka=tuple(m.Ka), Ks=tuple(m.Ks), Ns=m.Ns, Ni=m.Ni, Tr=m.Tr,
                    illum=m.illum, flags=m.flags)

    # -- hot path ----------------------------------------------------------------------------
    def intersect_mesh(self, origins, dests):
        """Batched intersectMesh: returns (index[n] int32, point[n,3] float32)."""
        o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(dests, np.float32).reshape(-1, 3)
        n = len(o)
        idx = np.zeros(n, np.int32)
        pts = np.zeros((n, 3), np.float32)
        check(lib().rt_intersect_mesh(self._h, _ptr(o), _ptr(d), n, _ptr(idx), _ptr(pts)))
        return idx, pts

    def perform_ray_tracing(self, params: RenderParams, origins, dests):
        """Batched performRayTracing: returns (rgb[n,3] float32 unclamped, counts[3])."""
        o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(dests, np.float32).reshape(-1, 3)
        n = len(o)
        rgb = np.zeros((n, 3), np.float32)
        counts = np.zeros(3, np.uint64)
        p = params.to_c()
        check(lib().rt_trace_rays(self._h, C.byref(p), _ptr(o), _ptr(d), n, _ptr(rgb), _ptr(counts)))
        return rgb, counts

    def debug_trace(self, params: RenderParams, origin, dest, max_bounces: int = 256):
        """The debug key 'd' (raytracing.cpp:493-510) for one ray: (bounces, rgb). Each bounce is
        a dict (origin, dest, hit, triangle, level, shadowed, lit) for one trace() call, in
        order; rgb = performRayTracing(origin, dest)."""
        from ._capi import RtDebugBounce
        buf = (RtDebugBounce * max_bounces)()
        n = C.c_int32()
        rgb = np.zeros(3, np.float32)
        o = np.ascontiguousarray(origin, np.float32).reshape(3)
        d = np.ascontiguousarray(dest, np.float32).reshape(3)
        p = params.to_c()
        check(lib().rt_debug_trace(self._h, C.byref(p), _ptr(o), _ptr(d), buf, max_bounces, C.byref(n), _ptr(rgb)))
        out = []
        for b in buf[: min(n.value, max_bounces)]:
            out.append(dict(origin=np.array(b.origin[:], np.float32), dest=np.array(b.dest[:], np.float32),
                            hit=np.array(b.hit[:], np.float32), triangle=b.triangle, level=b.level,
                            shadowed=b.shadowed, lit=b.lit))
        return out, rgb

    def render(self, params: RenderParams, x0: int = 0, y0: int = 0, w: int | None = None, h: int | None = None,
               want_f32: bool = False):
        """The 'r' key for a pixel rectangle: returns (u8[h,w,3], f32[h,w,3] or None, counts[3])."""
        w = params.width - x0 if w is None else w
        h = params.height - y0 if h is None else h
        u8 = np.zeros((h, w, 3), np.uint8)
        f32 = np.zeros((h, w, 3), np.float32) if want_f32 else None
        counts = np.zeros(3, np.uint64)
        p = params.to_c()
        check(lib().rt_render_tile(self._h, C.byref(p), x0, y0, w, h, _ptr(u8), _ptr(f32), _ptr(counts)))
        return u8, f32, counts

    def trace_frame_samples(self, params: RenderParams, with_rays: bool = False):
        """rt_trace_frame_samples: performRayTracing of every sub-sample of the 'r' loop (main.cpp:369-388),
        unclamped, in the loop's call order: rec[height, width, pfx, pfy, 3] float32 (the colour), or with
        with_rays [..., 9] (origin, dest, colour); and counts[3]."""
        pfy = params.pf if params.pfy is None else params.pfy
        layout = _capi.SAMPLES_RAY_RGB if with_rays else _capi.SAMPLES_RGB
        rec = np.zeros((params.height, params.width, params.pf, pfy, layout), np.float32)
        counts = np.zeros(3, np.uint64)
        p = params.to_c()
        check(lib().rt_trace_frame_samples(self._h, C.byref(p), layout, _ptr(rec), rec.size, _ptr(counts)))
        return rec, counts

    def render_frames_device(self, params: Sequence[RenderParams | RtParams], tile_w: int, tile_h: int, out_ptrs: Sequence[int],
                             out_capacity: int, stream_ptr: int | None = None, want_counts: bool = False):
        """rt_render_frames_device: len(params) views of one frame geometry (params differ in corners only),
        view f row-major into the device buffer out_ptrs[f], in one chain launch where possible."""
        n = len(params)
        if len(out_ptrs) != n:
            raise ValueError(f"render_frames_device: {n} views but {len(out_ptrs)} output buffers")
        arr = (RtParams * n)()
        keep = []
        for i, q in enumerate(params):
            c = q.to_c() if isinstance(q, RenderParams) else q
            keep.append(c)
            arr[i] = c
        outs = (C.c_void_p * n)(*[C.c_void_p(x) for x in out_ptrs])
        counts = np.zeros(3, np.uint64) if want_counts else None
        check(lib().rt_render_frames_device(self._h, arr, n, tile_w, tile_h, outs, out_capacity,
                                            C.c_void_p(stream_ptr) if stream_ptr else None, _ptr(counts)))
        return counts

    def reserve(self, params: RenderParams | RtParams, tile_w: int = 16, tile_h: int = 16, samples_layout: int = 0):
        """rt_scene_reserve: allocate what a frame of params needs (workspaces, sample staging) now,
        so its first render allocates nothing."""
        p = params.to_c() if isinstance(params, RenderParams) else params
        check(lib().rt_scene_reserve(self._h, C.byref(p), tile_w, tile_h, samples_layout))

    def render_tiles_device(self, params: RenderParams | RtParams, tile_w: int, tile_h: int, first: int, stride: int,
                            out_ptr: int, out_capacity: int, stream_ptr: int | None = None, want_counts: bool = False,
                            frames: int = 1):
        """Interleaved tile shard (ids first, first+stride, ... over `frames` frames of this view) into a
        device buffer, e.g. a torch uint8 CUDA tensor's data_ptr()."""
        p = params.to_c() if isinstance(params, RenderParams) else params
        n_tiles = C.c_int32()
        counts = np.zeros(3, np.uint64) if want_counts else None
        check(lib().rt_render_tiles_device(self._h, C.byref(p), tile_w, tile_h, frames, first, stride, C.c_void_p(out_ptr),
                                           out_capacity, C.c_void_p(stream_ptr) if stream_ptr else None,
                                           C.byref(n_tiles), _ptr(counts)))
        return n_tiles.value, counts

    def render_frame_device(self, params: RenderParams | RtParams, tile_w: int, tile_h: int, out_ptr: int,
                            out_capacity: int, stream_ptr: int | None = None, want_counts: bool = False):
        """The whole frame, row-major H x W x 3 bytes, into a device buffer (rt_render_frame_device)."""
        p = params.to_c() if isinstance(params, RenderParams) else params
        counts = np.zeros(3, np.uint64) if want_counts else None
        check(lib().rt_render_frame_device(self._h, C.byref(p), tile_w, tile_h, C.c_void_p(out_ptr), out_capacity,
                                           C.c_void_p(stream_ptr) if stream_ptr else None, _ptr(counts)))
        return counts

    def render_frames_sharded(self, params: RenderParams | RtParams, comm: "Comm", tile_w: int, tile_h: int, frames: int,
                              out_ptr: int | None, out_capacity: int, stream_ptr: int | None = None,
                              want_counts: bool = False):
        """rt_render_frames_sharded: this rank's interleaved tiles, one RCCL gather to rank 0 and the
        device un-permute there into out_ptr (frames x H x W x 3 bytes; rank 0 only)."""
        p = params.to_c() if isinstance(params, RenderParams) else params
        counts = np.zeros(3, np.uint64) if want_counts else None
        check(lib().rt_render_frames_sharded(self._h, C.byref(p), comm.handle, tile_w, tile_h, frames,
                                             C.c_void_p(out_ptr) if out_ptr else None, out_capacity,
                                             C.c_void_p(stream_ptr) if stream_ptr else None, _ptr(counts)))
        return counts

    # -- acceleration ------------------------------------------------------------------------
    def set_accel(self, mode) -> None:
        """'bvh' / 'brute_force' (or RT_ACCEL_* ints). Results are identical either way."""
        m = {"bvh": _capi.ACCEL_BVH, "brute_force": _capi.ACCEL_BRUTE_FORCE}.get(mode, mode)
        check(lib().rt_scene_set_accel(self._h, int(m)))

    def accel(self) -> str:
        m = C.c_int32()
        check(lib().rt_scene_get_accel(self._h, C.byref(m)))
        return "bvh" if m.value == _capi.ACCEL_BVH else "brute_force"

    def bvh_info(self) -> dict:
        info = np.zeros(_capi.BVH_INFO_FIELDS, np.int32)
        check(lib().rt_scene_bvh_info(self._h, _ptr(info)))
        return dict(nodes=int(info[0]), depth=int(info[1]), always=int(info[2]), never=int(info[3]),
                    leaf_triangles=int(info[4]), nodes4=int(info[5]), depth4=int(info[6]))

    def tune(self, knob: str, value: int) -> None:
        """Launch-shape knobs ('xcd_split', 'bvh_grid', 'bvh_width', 'lds_stack', 'pipes',
        'shadow_virtual', 'pipe_batches', 'pipe_priority', 'chain_from', 'chain_split', 'top_nodes',
        'batch_order', 'order_every', 'fuse_pixels', 'wave_steal', 'steal_half', 'steal_quarter',
        'cold_estimate', 'forget_order', 'split_eighth', 'prio_batches', 'pixel_order', 'dyn_group',
        'shadow_helpers', 'frames_in_flight';
        retired, 0 only: 'wave_traversal', 'chain_refill', 'refill_grid'); outputs never depend on
        them."""
        k = {"xcd_split": _capi.TUNE_XCD_SPLIT, "bvh_grid": _capi.TUNE_BVH_GRID,
             "bvh_width": _capi.TUNE_BVH_WIDTH, "lds_stack": _capi.TUNE_LDS_STACK,
             "pipes": _capi.TUNE_PIPES, "shadow_virtual": _capi.TUNE_SHADOW_VIRTUAL,
             "pipe_batches": _capi.TUNE_PIPE_BATCHES, "pipe_priority": _capi.TUNE_PIPE_PRIORITY,
             "wave_traversal": _capi.TUNE_WAVE_TRAVERSAL, "chain_from": _capi.TUNE_CHAIN_FROM,
             "chain_split": _capi.TUNE_CHAIN_SPLIT, "top_nodes": _capi.TUNE_TOP_NODES,
             "batch_order": _capi.TUNE_BATCH_ORDER,
             "order_every": _capi.TUNE_ORDER_EVERY, "fuse_pixels": _capi.TUNE_FUSE_PIXELS,
             "chain_refill": _capi.TUNE_CHAIN_REFILL, "refill_grid": _capi.TUNE_REFILL_GRID,
             "wave_steal": _capi.TUNE_WAVE_STEAL, "steal_half": _capi.TUNE_STEAL_HALF,
             "steal_quarter": _capi.TUNE_STEAL_QUARTER, "cold_estimate": _capi.TUNE_COLD_ESTIMATE,
             "forget_order": _capi.TUNE_FORGET_ORDER, "split_eighth": _capi.TUNE_SPLIT_EIGHTH,
             "prio_batches": _capi.TUNE_PRIORITY_BATCHES,
             "pixel_order": _capi.TUNE_PIXEL_ORDER, "dyn_group": _capi.TUNE_DYN_GROUP,
             "shadow_helpers": _capi.TUNE_SHADOW_HELPERS, "frames_in_flight": _capi.TUNE_FRAMES_IN_FLIGHT,
             "adopt_order": _capi.TUNE_ADOPT_ORDER, "inflight_dynamic": _capi.TUNE_INFLIGHT_DYNAMIC,
             "inflight_streams": _capi.TUNE_INFLIGHT_STREAMS, "quad_walk": _capi.TUNE_QUAD_WALK,
             "motion_order": _capi.TUNE_MOTION_ORDER, "order_early": _capi.TUNE_ORDER_EARLY}[knob]
        check(lib().rt_scene_tune(self._h, k, int(value)))

    def workspace_bytes(self) -> tuple[int, int]:
        """rt_workspace_bytes: (bytes of the render workspaces held now, multi-frame calls that fell back to
        rendering frame by frame)."""
        b, f = C.c_uint64(), C.c_uint64()
        check(lib().rt_workspace_bytes(self._h, C.byref(b), C.byref(f)))
        return b.value, f.value

    def trials(self) -> dict:
        """rt_scene_trials: the per-view launch trials (steal x distribution x shadow helpers) of
        pipeline 0."""
        info = np.zeros(_capi.RT_TRIAL_INFO_FIELDS, np.int32)
        ms = np.zeros(_capi.RT_MAX_TRIALS, np.float32)
        check(lib().rt_scene_trials(self._h, info.ctypes.data, ms.ctypes.data))
        n = int(info[0])
        return {"trials": n, "choice": int(info[1]), "wave_steal": int(info[2]), "chain_split": int(info[3]),
                "shadow_helpers": int(info[4]), "steal_quarter": int(info[5]), "inflight_split": int(info[6]),
                "trial_ms": [round(float(x), 4) for x in ms[:n]]}

    def batch_durations(self) -> np.ndarray:
        """Per wave batch of the latest chain launch: the wave's duration in microseconds
        (rt_batch_durations; 100 MHz ticks). Its maximum is the launch's critical path."""
        n = C.c_int64()
        check(lib().rt_batch_durations(self._h, None, 0, C.byref(n)))
        out = np.zeros(n.value, np.uint32)
        if n.value:
            check(lib().rt_batch_durations(self._h, out.ctypes.data, n.value, C.byref(n)))
        return out.astype(np.float64) * 0.01

    def bvh_digest(self) -> int:
        """FNV-1a digest of the device BVH arrays (identical trees <=> equal digests)."""
        d = C.c_uint64()
        check(lib().rt_scene_bvh_digest(self._h, C.byref(d)))
        return d.value

    def bvh_validate(self) -> None:
        check(lib().rt_scene_bvh_validate(self._h))

    # -- measurement -------------------------------------------------------------------------
    def set_profiling(self, enabled: bool | int, count_work: bool = False) -> None:
        """Time every launch (HIP events); with count_work the BVH kernels also count their work
        (rt_work_detail), which slows them: time and count in separate passes."""
        mode = 0 if not enabled else (2 if count_work else 1)
        check(lib().rt_set_profiling(self._h, mode))

    def kernel_stats(self, kind: int) -> tuple[int, float, float]:
        launches, ms, tests = C.c_uint64(), C.c_double(), C.c_double()
        check(lib().rt_kernel_stats(self._h, kind, C.byref(launches), C.byref(ms), C.byref(tests)))
        return launches.value, ms.value, tests.value

    def reset_stats(self) -> None:
        check(lib().rt_reset_stats(self._h))

    def work_stats(self, kind: int = _capi.KERNEL_CLOSEST_HIT) -> tuple[float, float]:
        """(ray-triangle tests, BVH node visits) executed by the BVH kernels of `kind` since
        reset_stats()."""
        t, v = C.c_double(), C.c_double()
        check(lib().rt_work_stats(self._h, kind, C.byref(t), C.byref(v)))
        return t.value, v.value

    def diag_read(self, offset: int, count: int) -> np.ndarray:
        """Diagnostic words of a diagnostic kernel build (rt_diag_read)."""
        d = np.zeros(count, np.uint64)
        check(lib().rt_diag_read(self._h, offset, count, _ptr(d)))
        return d

    def work_detail(self, kind: int = _capi.KERNEL_CLOSEST_HIT) -> dict:
        """Full BVH work counters of `kind` (rt_work_detail): tests, visits, the per-wave-task
        maxima that give the traversal's SIMD efficiency, the longest query."""
        d = np.zeros(_capi.WORK_FIELDS, np.uint64)
        check(lib().rt_work_detail(self._h, kind, _ptr(d)))
        keys = ("tests", "visits", "wave_max_visits", "max_visits", "wave_tasks", "wave_max_tests")
        out = {k: int(x) for k, x in zip(keys, d)}
        out["simd_eff_visits"] = out["visits"] / max(1, 64 * out["wave_max_visits"])
        out["simd_eff_tests"] = out["tests"] / max(1, 64 * out["wave_max_tests"])
        return out


def load_mtl(path: str) -> list[tuple[str, dict]]:
    """rt_load_mtl: every block Mesh::loadMtl would commit from one MTL file, in file order, as
    (name, material); the caller keeps the first block of each name not already indexed."""
    n = C.c_int32()
    check(lib().rt_load_mtl(path.encode(), C.byref(n), None, 0, None, 0))
    mats = (RtMaterial * max(n.value, 1))()
    cap = 1
    with open(path, "rb") as f:   # (names are at most the file's bytes)
        cap += len(f.read()) + n.value
    names = C.create_string_buffer(cap)
    check(lib().rt_load_mtl(path.encode(), C.byref(n), C.cast(mats, C.c_void_p), n.value, names, cap))
    raw = names.raw.split(b"\0")[: n.value]
    return [(nm.decode(), dict(Kd=tuple(m.Kd), Ka=tuple(m.Ka), Ks=tuple(m.Ks), Ns=m.Ns, Ni=m.Ni, Tr=m.Tr,
                               illum=m.illum, flags=m.flags)) for nm, m in zip(raw, list(mats)[: n.value])]


def bvh_acceptance_box(T) -> tuple[int, np.ndarray, np.ndarray]:
    """(status, lo, hi) of the BVH's padded acceptance box for triangle T (3x3): status 0 = box,
    1 = ill-conditioned (tested by every query), 2 = never accepted (n == 0)."""
    t = np.ascontiguousarray(T, np.float32).reshape(9)
    lo = np.zeros(3, np.float32)
    hi = np.zeros(3, np.float32)
    st = lib().rt_bvh_acceptance_box(_ptr(t), _ptr(lo), _ptr(hi))
    if st < 0:
        check(st)
    return st, lo, hi


class Comm:
    """An RCCL communicator of the library (rt_comm_*): one rank per GPU. Rank 0 calls
    Comm.unique_id() and hands the bytes to every rank, which then constructs Comm(...)."""

    def __init__(self, device: int, rank: int, nranks: int, uid: bytes):
        if len(uid) != _capi.COMM_ID_BYTES:
            raise ValueError("communicator id must be 128 bytes")
        buf = (C.c_uint8 * _capi.COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib().rt_comm_init(device, rank, nranks, buf, C.byref(h)))
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * _capi.COMM_ID_BYTES)()
        check(lib().rt_comm_unique_id(buf))
        return bytes(buf)

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def info(self) -> tuple[int, int, int]:
        r, n, d = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib().rt_comm_info(self._h, C.byref(r), C.byref(n), C.byref(d)))
        return r.value, n.value, d.value

    def check(self) -> None:
        check(lib().rt_comm_check(self._h))

    def set_pipeline(self, depth: int) -> None:
        """rt_comm_set_pipeline: 2 overlaps each call's render with the previous call's gather and
        un-permute (collective; every rank sets the same depth)."""
        check(lib().rt_comm_set_pipeline(self._h, depth))

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().rt_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def assemble_tiles_device(device: int, width: int, height: int, tile_w: int, tile_h: int, frames: int, nranks: int,
                          gathered_ptr: int, gathered_bytes: int, out_ptr: int, out_capacity: int,
                          stream_ptr: int | None = None) -> None:
    """rt_assemble_tiles_device: un-permute gathered tile shards into frames x H x W x 3 bytes."""
    check(lib().rt_assemble_tiles_device(device, width, height, tile_w, tile_h, frames, nranks, C.c_void_p(gathered_ptr),
                                         gathered_bytes, C.c_void_p(out_ptr), out_capacity,
                                         C.c_void_p(stream_ptr) if stream_ptr else None))


def ray_intersect_triangle(rays, tris, device: int = 0):
    """rayIntersectTriangle (raytracing.cpp:99-154) for n (ray, triangle) pairs on the GPU:
    rays [n, 2, 3] (origin, dest), tris [n, 3, 3] -> (hit[n] bool, point[n, 3] float32)."""
    R_ = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    T_ = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    if len(R_) != len(T_):
        raise ValueError("rays and tris differ in length")
    n = len(R_)
    hit = np.zeros(n, np.uint8)
    pts = np.zeros((n, 3), np.float32)
    check(lib().rt_ray_intersect_triangle(device, _ptr(R_), _ptr(T_), n, _ptr(hit), _ptr(pts)))
    return hit.astype(bool), pts


def device_count() -> int:
    n = C.c_int32()
    check(lib().rt_device_count(C.byref(n)))
    return n.value


__all__ = ["Scene", "RenderParams", "Comm", "default_corners", "write_ppm", "device_count", "ray_intersect_triangle",
           "assemble_tiles_device", "RT_HOST_ONLY"]
