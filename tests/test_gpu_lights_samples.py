"""GPU parity for the r04 boundary additions, against the oracle.

* Any number of lights (VERDICT r03 "What's missing" 1): the reference's MyLightPositions is an
  unbounded std::vector (raytracing.h:9) that 'L' grows (main.cpp:334-336) and shade() loops over
  in order (raytracing.cpp:342-356). rt_params.light_list carries more than RT_MAX_LIGHTS (16);
  up to 16 run in the chain launch (from its arguments), 17 and more in the per-step kernels (r04;
  r03-r04 ran 17-32 in the chain launch). Whole frames with 17, 32, 33 and 64 lights equal the oracle's, on the opaque and the
  transparent sphere grids and on dodgeColorTest; rt_trace_rays and the debug trace too.
* rt_trace_frame_samples: every sub-sample of the 'r' loop (main.cpp:369-388) in the loop's call
  order, with the ray the device made for it. The rays equal the loop's binary32 expressions
  (main.cpp:380-386, restated in numpy float32) bit for bit; each pixel's sub-samples, summed in
  the loop's order, divided and clamped, equal the oracle's frame floats bit for bit; sampled
  sub-samples equal the oracle's performRayTracing of the same ray.
* rt_batch_durations after rt_trace_rays grew the workspace; rt_trace_rays between
  ordered frames leaves the frames unchanged.
"""
import numpy as np
import pytest

import oracle as O
import raytracert_amd as R
from _util import scene_path

pytestmark = pytest.mark.gpu

ORACLE_THREADS = 16


def _lights(n):
    """n distinct lights around the scene (deterministic): a spiral in front of the spheres."""
    t = np.arange(n, dtype=np.float64)
    return [(float(np.float32(1.6 * np.cos(0.7 * i))), float(np.float32(1.2 * np.sin(0.7 * i))),
             float(np.float32(2.5 + 0.03 * i))) for i in t]


@pytest.mark.parametrize("n_lights", [17, 32, 33, 64])
@pytest.mark.parametrize("spec,w,h,pf,max_lvl", [("syn:F3", 96, 54, 1, 3), ("syn:F4", 64, 36, 2, 4),
                                                 ("ref:dodgeColorTest.obj", 80, 60, 1, 2)])
def test_more_lights_than_inline_full_frame(spec, w, h, pf, max_lvl, n_lights, workdir, gpu_available):
    path = scene_path(spec, workdir)
    lights = _lights(n_lights)
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=max_lvl, lights=lights)
    with R.Scene.load(path, device=0) as sc:
        u8, f32, counts = sc.render(p, want_f32=True)
        u8b, _, _ = sc.render(p, want_f32=False)   # (second call: the device list is not re-uploaded)
    of32, ou8, oc = O.OracleScene(path).render(O.make_params(w, h, pf, max_lvl, lights=lights), nthreads=ORACLE_THREADS)
    assert [int(c) for c in counts] == [int(c) for c in oc]
    assert int(oc[2]) > 0
    assert np.array_equal(u8, ou8) and np.array_equal(u8b, ou8)
    assert np.array_equal(f32.view(np.uint32), of32.view(np.uint32))


def test_light_list_changes_between_frames(workdir, gpu_available):
    """The device copy of a light list follows every change (same count, other positions; a longer
    list; back to inline), frame after frame on one scene."""
    path = scene_path("syn:F3", workdir)
    orc = O.OracleScene(path)
    w, h = 64, 36
    with R.Scene.load(path, device=0) as sc:
        for lights in (_lights(20), [tuple(np.float32(v) * np.float32(0.9) for v in l) for l in _lights(20)],
                       _lights(40), _lights(3), _lights(20)):
            p = R.RenderParams(width=w, height=h, pf=1, max_lvl=2, lights=lights)
            u8, _, counts = sc.render(p)
            _, ou8, oc = orc.render(O.make_params(w, h, 1, 2, lights=lights), nthreads=ORACLE_THREADS)
            assert [int(c) for c in counts] == [int(c) for c in oc]
            assert np.array_equal(u8, ou8)


@pytest.mark.parametrize("n_lights", [20, 40])
def test_more_lights_trace_rays_and_debug_trace(n_lights, workdir, gpu_available):
    """performRayTracing (rt_trace_rays, the per-step kernels at any light count) and the debug key's
    records with more than 16 lights; the records' shadow masks hold lights 0-31."""
    path = scene_path("syn:F4", workdir)
    orc = O.OracleScene(path)
    lights = _lights(n_lights)
    p = R.RenderParams(width=64, height=36, pf=1, max_lvl=4, lights=lights)
    op = O.make_params(64, 36, 1, 4, lights=lights)
    cs = R.default_corners(64, 36)
    rng = np.random.default_rng(7)
    t = rng.random((48, 2)).astype(np.float32)
    orgs = (cs[0] * (1 - t[:, :1]) + cs[6] * t[:, :1]).astype(np.float32)
    dsts = (cs[1] * (1 - t[:, 1:]) + cs[7] * t[:, 1:]).astype(np.float32)
    with R.Scene.load(path, device=0) as sc:
        rgb, _ = sc.perform_ray_tracing(p, orgs, dsts)
        for i in range(len(orgs)):
            orgb, _ = orc.trace(op, orgs[i], dsts[i])
            assert np.array_equal(rgb[i].view(np.uint32), orgb.view(np.uint32)), i
        for i in range(0, len(orgs), 6):
            b, c = sc.debug_trace(p, orgs[i], dsts[i])
            ob, oc = orc.debug_trace(op, orgs[i], dsts[i])
            assert len(b) == len(ob)
            assert np.array_equal(c.view(np.uint32), oc.view(np.uint32))
            for x, y in zip(b, ob):
                assert x["triangle"] == y["triangle"] and x["shadowed"] == y["shadowed"] and x["lit"] == y["lit"]


def loop_rays(cs, w, h, pfx, pfy):
    """main.cpp:380-386 for every (y, x, subx, suby), in binary32 with the loop's operation order."""
    f = np.float32
    divX, divY = f(w * pfx - 1), f(h * pfy - 1)
    xs = (f(1) - (np.arange(w, dtype=f)[:, None] * f(pfx) + np.arange(pfx, dtype=f)[None, :]) / divX).reshape(-1)
    ys = (f(1) - (np.arange(h, dtype=f)[:, None] * f(pfy) + np.arange(pfy, dtype=f)[None, :]) / divY).reshape(-1)
    X = xs[None, :, None]   # [1, cols, 1]
    Y = ys[:, None, None]   # [rows, 1, 1]
    out = []
    for a, b, c, d in ((0, 4, 2, 6), (1, 5, 3, 7)):
        A = X * cs[a] + (f(1) - X) * cs[b]
        B = X * cs[c] + (f(1) - X) * cs[d]
        out.append(Y * A + (f(1) - Y) * B)   # [rows, cols, 3]
    o, dd = out
    # rows = y * pfy + suby, cols = x * pfx + subx -> [h, w, pfx, pfy, 3]
    def reorder(v):
        return v.reshape(h, pfy, w, pfx, 3).transpose(0, 2, 3, 1, 4)
    return reorder(o), reorder(dd)


@pytest.mark.parametrize("spec,w,h,pf,max_lvl,nl", [("ref:dodgeColorTest.obj", 100, 80, 3, 10, 1),
                                                    ("syn:F4", 64, 36, 2, 4, 2), ("syn:C4", 96, 54, 1, 3, 2),
                                                    ("syn:F3", 48, 27, 9, 3, 20)])
def test_trace_frame_samples_match_loop_and_oracle(spec, w, h, pf, max_lvl, nl, workdir, gpu_available):
    """Records of rt_trace_frame_samples: rays = the loop's (bitwise); per-pixel ordered sums / spp,
    clamped = the oracle frame (bitwise); sampled colours = the oracle's trace of the same ray; the
    colour-only layout = the colours of the ray layout; ray counts = the frame's. pf 9 (81 sub-samples
    per pixel) takes the unfused path, 20 lights the per-step kernels with the device light list."""
    path = scene_path(spec, workdir)
    lights = _lights(nl) if nl > 2 else [(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)][:nl]
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=max_lvl, lights=lights)
    op = O.make_params(w, h, pf, max_lvl, lights=lights)
    orc = O.OracleScene(path)
    with R.Scene.load(path, device=0) as sc:
        rec, counts = sc.trace_frame_samples(p, with_rays=True)
        rgb_only, counts2 = sc.trace_frame_samples(p)
        _, _, fcounts = sc.render(p)
    assert rec.shape == (h, w, pf, pf, 9)
    lo, ld = loop_rays(R.default_corners(w, h), w, h, pf, pf)
    assert np.array_equal(rec[..., 0:3].view(np.uint32), lo.view(np.uint32))
    assert np.array_equal(rec[..., 3:6].view(np.uint32), ld.view(np.uint32))
    col = rec[..., 6:9]
    assert np.array_equal(col.view(np.uint32), rgb_only.view(np.uint32))
    assert [int(c) for c in counts] == [int(c) for c in fcounts] == [int(c) for c in counts2]
    # the loop's per-pixel sum (subx outer, suby inner), rgb / raysPerPixel, RGBValue clamp
    acc = np.zeros((h, w, 3), np.float32)
    for sx in range(pf):
        for sy in range(pf):
            acc = acc + col[:, :, sx, sy]
    acc = acc / np.float32(pf * pf)
    acc = np.where(acc > 1, np.float32(1), acc)
    acc = np.where(acc < 0, np.float32(0), acc)
    of32, _, _ = orc.render(op, nthreads=ORACLE_THREADS)
    assert np.array_equal(acc.view(np.uint32), of32.view(np.uint32))
    rng = np.random.default_rng(3)
    for _ in range(24):
        y, x, sx, sy = rng.integers(h), rng.integers(w), rng.integers(pf), rng.integers(pf)
        orgb, _ = orc.trace(op, lo[y, x, sx, sy], ld[y, x, sx, sy])
        assert np.array_equal(col[y, x, sx, sy].view(np.uint32), orgb.view(np.uint32)), (y, x, sx, sy)


def test_trace_frame_samples_arguments(workdir, gpu_available):
    from raytracert_amd import _capi
    import ctypes as C
    with R.Scene.load(scene_path("syn:F3", workdir), device=0) as sc:
        p = R.RenderParams(width=8, height=4, pf=2, max_lvl=1).to_c()
        small = np.zeros(8 * 4 * 4 * 3 - 1, np.float32)
        for layout, buf in ((3, small), (7, np.zeros(8 * 4 * 4 * 9, np.float32))):
            rc = _capi.lib().rt_trace_frame_samples(sc.handle, C.byref(p), layout, buf.ctypes.data, buf.size, None)
            assert rc == _capi.RT_E_ARG


def test_batch_durations_after_trace_rays_grows_workspace(workdir, gpu_available):
    """rt_trace_rays with more rays than the frame reallocates pipeline 0's
    workspace; rt_batch_durations afterwards must not read the freed cost buffer: it reports no batches
    until the next chain launch measures some, then that launch's."""
    p = R.RenderParams(width=64, height=48, pf=1, max_lvl=2, lights=[(0.0, 0.0, 4.0)])
    with R.Scene.load(scene_path("syn:F3", workdir), device=0) as sc:
        sc.render(p)
        assert sc.batch_durations().size == (64 * 48 + 63) // 64
        n = 200_000
        cs = R.default_corners(64, 48)
        t = np.linspace(0, 1, n, dtype=np.float32)[:, None]
        sc.perform_ray_tracing(p, cs[0] * (1 - t) + cs[6] * t, cs[1] * (1 - t) + cs[7] * t)
        assert sc.batch_durations().size == 0
        sc.render(p)
        d = sc.batch_durations()
        assert d.size == (64 * 48 + 63) // 64 and np.all(d > 0) and np.all(d < 1e6)


def test_trace_rays_between_ordered_frames_keeps_frames(workdir, gpu_available):
    """rt_trace_rays between ordered renders of a view writes no batch
    durations (its launch has no pipeline order), so the re-sorts that follow see only the frames'
    own durations; every frame stays byte-identical."""
    p = R.RenderParams(width=320, height=180, pf=1, max_lvl=3, lights=[(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)])
    with R.Scene.load(scene_path("syn:C4", workdir), device=0) as sc:
        sc.tune("order_every", 1)
        ref, _, cref = sc.render(p)
        cs = R.default_corners(320, 180)
        t = np.linspace(0, 1, 50_000, dtype=np.float32)[:, None]
        for i in range(6):
            sc.perform_ray_tracing(p, cs[0] * (1 - t) + cs[6] * t, cs[1] * (1 - t) + cs[7] * t)
            u8, _, c = sc.render(p)
            assert np.array_equal(u8, ref) and [int(x) for x in c] == [int(x) for x in cref], i
