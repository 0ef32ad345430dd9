"""GPU parity: librtamd.so on cuda:0 against the oracle and the committed golden fixtures.

Bar (north_star): PPM bytes within 1 LSB per channel of the CPU reference; in practice the only
arithmetic that may differ is powf(SpecularTerm, Ns) (the GPU rounds a double pow once; glibc
powf is not always correctly rounded), which is colour-only. Every hit/miss decision, hit index
and hit point is compared bit for bit, and so are the per-kind ray counts.
"""
import numpy as np
import pytest

import oracle as O
import raytracert_amd as R
from _util import golden, golden_index, scene_path, survey_pins

pytestmark = pytest.mark.gpu

LSB_TOL = 1            # per-channel |delta| allowed on 8-bit output (north_star)
F32_TOL = 2e-6         # float RGB tolerance (colour-only powf rounding)
EXACT_FRAC = 0.9999    # fraction of bytes that must be bit-identical


def _params(entry):
    return R.RenderParams(width=entry["width"], height=entry["height"], pf=entry["pf"], max_lvl=entry["max_lvl"],
                          lights=entry["lights"])


def _assert_image_close(u8, f32, gu8, gf32):
    d = np.abs(u8.astype(np.int16) - gu8.astype(np.int16))
    assert d.max() <= LSB_TOL, f"max byte delta {d.max()}"
    assert (d == 0).mean() >= EXACT_FRAC, f"exact bytes {(d == 0).mean():.6f}"
    if f32 is not None:
        assert np.abs(f32 - gf32).max() <= F32_TOL


@pytest.mark.parametrize("name", sorted(golden_index()))
def test_render_matches_golden(name, workdir, gpu_available):
    entry = golden_index()[name]
    gu8, gf32 = golden(name)
    with R.Scene.load(scene_path(entry["scene"], workdir), device=0) as sc:
        u8, f32, counts = sc.render(_params(entry), want_f32=True)
    assert [int(c) for c in counts] == entry["counts"]
    _assert_image_close(u8, f32, gu8, gf32)


def test_c2_full_frame_counts_and_bytes(workdir, gpu_available):
    pin = survey_pins()["C2"]
    path = scene_path("ref:dodgeColorTest.obj", workdir)
    p = R.RenderParams(width=800, height=600, pf=1, max_lvl=1, lights=pin["lights"])
    with R.Scene.load(path, device=0) as sc:
        u8, f32, counts = sc.render(p, want_f32=True)
    assert [int(c) for c in counts] == [pin["rays_primary"], pin["rays_secondary"], pin["rays_shadow"]]
    o = O.OracleScene(path)
    of32, ou8, ocounts = o.render(O.make_params(800, 600, 1, 1, lights=pin["lights"]), nthreads=16)
    assert [int(c) for c in ocounts] == [int(c) for c in counts]
    _assert_image_close(u8, f32, ou8, of32)


def test_c4_48x27_ray_count(workdir, gpu_available):
    pin = survey_pins()["C4_48x27"]
    with R.Scene.load(scene_path("syn:C4", workdir), device=0) as sc:
        _, _, counts = sc.render(R.RenderParams(width=48, height=27, pf=1, max_lvl=3, lights=pin["lights"]))
    assert int(counts.sum()) == pin["rays_total"]


def test_c4_tiles_at_full_resolution(workdir, gpu_available):
    """F7: 32x32 tiles of the C4 frame at 1920x1080 (centre, sphere edge, corner) vs the oracle."""
    path = scene_path("syn:C4", workdir)
    lights = [[0, 0, 4], [1.5, 1.5, 4]]
    p = R.RenderParams(width=1920, height=1080, pf=1, max_lvl=3, lights=lights)
    op = O.make_params(1920, 1080, 1, 3, lights=lights)
    o = O.OracleScene(path)
    with R.Scene.load(path, device=0) as sc:
        for x0, y0 in [(944, 524), (700, 300), (0, 0), (1888, 1048)]:
            u8, f32, counts = sc.render(p, x0, y0, 32, 32, want_f32=True)
            of32, ou8, oc = o.render(op, x0, y0, 32, 32, nthreads=16)
            assert [int(c) for c in counts] == [int(c) for c in oc]
            _assert_image_close(u8, f32, ou8, of32)


def test_intersect_mesh_bitwise(workdir, gpu_available):
    """Batched intersectMesh: index and hit point bit-identical to the oracle for primary-like,
    random and grazing rays, including ties between duplicated triangles."""
    path = scene_path("ref:dodgeColorTest.obj", workdir)
    o = O.OracleScene(path)
    rng = np.random.default_rng(7)
    n = 600
    c = R.default_corners(200, 150)
    t = rng.random((n, 2)).astype(np.float32)
    org = (c[0] * (1 - t[:, :1]) + c[6] * t[:, :1]).astype(np.float32)
    dst = (c[1] * (1 - t[:, 1:]) + c[7] * t[:, 1:]).astype(np.float32)
    rnd_o = (rng.standard_normal((n, 3)) * 0.5).astype(np.float32)
    rnd_d = (rng.standard_normal((n, 3)) * 0.5).astype(np.float32)
    origins = np.concatenate([org, rnd_o])
    dests = np.concatenate([dst, rnd_d])
    with R.Scene.load(path, device=0) as sc:
        idx, pts = sc.intersect_mesh(origins, dests)
    hits = 0
    for i in range(len(origins)):
        oi, opt = o.intersect_mesh(origins[i], dests[i])
        assert idx[i] == oi, i
        assert np.array_equal(pts[i].view(np.uint32), opt.view(np.uint32)), i
        hits += oi >= 0
    assert hits > 50


def test_perform_ray_tracing_batched(workdir, gpu_available):
    path = scene_path("syn:F4", workdir)
    o = O.OracleScene(path)
    lights = [[0, 0, 4], [1.5, 1.5, 4]]
    p = R.RenderParams(width=64, height=36, pf=1, max_lvl=6, lights=lights)
    op = O.make_params(64, 36, 1, 6, lights=lights)
    rng = np.random.default_rng(3)
    c = R.default_corners(64, 36)
    t = rng.random((500, 2)).astype(np.float32)
    origins = (c[0] * (1 - t[:, :1]) + c[6] * t[:, :1]).astype(np.float32)
    dests = (c[1] * (1 - t[:, 1:]) + c[7] * t[:, 1:]).astype(np.float32)
    with R.Scene.load(path, device=0) as sc:
        rgb, counts = sc.perform_ray_tracing(p, origins, dests)
    tot = np.zeros(3, np.uint64)
    for i in range(len(origins)):
        orgb, oc = o.trace(op, origins[i], dests[i])
        tot += oc
        assert np.abs(rgb[i] - orgb).max() <= F32_TOL, i
    assert [int(x) for x in counts] == [int(x) for x in tot]


def test_sharded_tiles_reassemble_to_full_frame(workdir, gpu_available):
    """rt_render_tiles_device with an interleaved stride reassembles to the rectangle render."""
    import torch
    path = scene_path("syn:F3", workdir)
    p = R.RenderParams(width=100, height=70, pf=2, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    from raytracert_amd import dist
    with R.Scene.load(path, device=0) as sc:
        full, _, counts = sc.render(p)
        layout = dist.TileLayout(p.width, p.height, 16, 16)
        parts = []
        total = np.zeros(3, np.uint64)
        for rank in range(3):
            buf = torch.zeros(layout.shard_bytes(3), dtype=torch.uint8, device="cuda:0")
            n, c = sc.render_tiles_device(p, 16, 16, rank, 3, buf.data_ptr(), buf.numel(),
                                          torch.cuda.current_stream().cuda_stream, want_counts=True)
            assert n == layout.tiles_of(rank, 3)
            total += c
            parts.append(buf.cpu().numpy())
        frame = layout.assemble(parts)
    assert np.array_equal(frame, full)
    assert [int(x) for x in total] == [int(x) for x in counts]


@pytest.mark.parametrize("size,pf", [((100, 70), 2), ((1920, 1080), 1)])
def test_frame_device_equals_rectangle_render(size, pf, workdir, gpu_available):
    """rt_render_frame_device (the single-GPU bench path) writes the row-major frame the rectangle
    render returns, with the same ray counts, twice in a row (the second launch batch-ordered)."""
    import torch
    w, h = size
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    with R.Scene.load(scene_path("syn:C4" if w > 1000 else "syn:F3", workdir), device=0) as sc:
        full, _, counts = sc.render(p)
        buf = torch.full((h * w * 3,), 7, dtype=torch.uint8, device="cuda:0")
        for _ in range(2):
            c = sc.render_frame_device(p, 16, 16, buf.data_ptr(), buf.numel(), torch.cuda.current_stream().cuda_stream,
                                       want_counts=True)
            assert np.array_equal(buf.view(h, w, 3).cpu().numpy(), full)
            assert [int(x) for x in c] == [int(x) for x in counts]


@pytest.mark.parametrize("spec,size,pf,want_f32", [("syn:F3", (100, 70), 1, True), ("syn:C4", (1920, 1080), 1, False),
                                                    ("syn:F4", (37, 23), 1, True), ("syn:F3", (100, 70), 2, True),
                                                    ("syn:F4", (37, 23), 4, True), ("syn:F3", (61, 29), 3, True),
                                                    ("syn:C4", (640, 360), 2, False)])
def test_fused_pixel_writes_equal_frame_pass(spec, size, pf, want_f32, workdir, gpu_available):
    """RT_TUNE_FUSE_PIXELS: the chain launch writes each pixel when its samples' chains end (the
    pf^2 sub-samples summed across adjacent lanes in k_frame's order; pf 3 packs 7 pixels into 63
    lanes, and its batch order must not be taken from the unfused launch's 64-query batches).
    Bytes, floats and ray counts equal the separate frame pass's, for
    the rectangle render, the whole-frame device render and the tile-major shard layout (whose
    pixels outside the frame are written black: ragged sizes leave partial tiles)."""
    import torch
    w, h = size
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    ntiles = ((w + 15) // 16) * ((h + 15) // 16)
    out = {}
    with R.Scene.load(scene_path(spec, workdir), device=0) as sc:
        for fuse in (0, 1):
            sc.tune("fuse_pixels", fuse)
            u8, f32, c = sc.render(p, want_f32=want_f32)
            fb = torch.full((h * w * 3,), 7, dtype=torch.uint8, device="cuda:0")
            sc.render_frame_device(p, 16, 16, fb.data_ptr(), fb.numel(), torch.cuda.current_stream().cuda_stream)
            tb = torch.full((ntiles * 256 * 3,), 7, dtype=torch.uint8, device="cuda:0")
            n, tc = sc.render_tiles_device(p, 16, 16, 0, 1, tb.data_ptr(), tb.numel(),
                                           torch.cuda.current_stream().cuda_stream, want_counts=True)
            assert n == ntiles
            out[fuse] = (u8, f32, [int(x) for x in c], fb.cpu().numpy(), tb.cpu().numpy(), [int(x) for x in tc])
    a, b = out[0], out[1]
    assert np.array_equal(a[0], b[0]) and a[2] == b[2] and a[5] == b[5]
    if want_f32:
        assert np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
    assert np.array_equal(a[3], b[3]) and np.array_equal(b[3].reshape(h, w, 3), b[0])
    assert np.array_equal(a[4], b[4])


@pytest.mark.parametrize("spec,size,pf,tile", [("syn:F3", (100, 70), 1, 16), ("syn:F3", (100, 70), 2, 16),
                                               ("syn:F3", (61, 29), 3, 16), ("syn:F4", (37, 23), 4, 8),
                                               ("syn:C4", (1920, 1080), 1, 16), ("syn:F3", (100, 70), 1, 32),
                                               ("syn:F3", (100, 70), 2, 12)])
def test_pixel_order_keeps_results(spec, size, pf, tile, workdir, gpu_available):
    """RT_TUNE_PIXEL_ORDER only changes which pixels share a wave batch: row-major, Morton (square
    power-of-two tiles; a 12x12 tile stays row-major) and auto give the same frame (the row-major
    device frame, the tile-major shard layout with its rows un-permuted as before, the rectangle
    render) and the same ray counts, cold and batch-ordered, with the fused frame and the frame pass."""
    import torch
    w, h = size
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    ntiles = ((w + tile - 1) // tile) * ((h + tile - 1) // tile)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    with R.Scene.load(scene_path(spec, workdir), device=0) as sc:
        for fuse in (1, 0):
            sc.tune("fuse_pixels", fuse)
            for order in (0, 1, 2):
                sc.tune("pixel_order", order)
                sc.tune("forget_order", 1)
                for rep in range(2):   # cold, then ordered by the first launch's durations
                    fb = torch.full((h * w * 3,), 7, dtype=torch.uint8, device="cuda:0")
                    c = sc.render_frame_device(p, tile, tile, fb.data_ptr(), fb.numel(), stream, want_counts=True)
                    tb = torch.full((ntiles * tile * tile * 3,), 7, dtype=torch.uint8, device="cuda:0")
                    n, tc = sc.render_tiles_device(p, tile, tile, 0, 1, tb.data_ptr(), tb.numel(), stream, want_counts=True)
                    assert n == ntiles
                    out[(fuse, order, rep)] = (fb.cpu().numpy(), tb.cpu().numpy(), [int(x) for x in c], [int(x) for x in tc])
        u8, _, counts = sc.render(p)
    ref = out[(0, 0, 0)]
    assert np.array_equal(ref[0].reshape(h, w, 3), u8) and ref[2] == [int(x) for x in counts]
    for key, v in out.items():
        assert np.array_equal(v[0], ref[0]), key
        assert np.array_equal(v[1], ref[1]), key
        assert v[2] == ref[2] and v[3] == ref[2], key


def test_transparent_shadow_path_and_deep_chain(workdir, gpu_available):
    """F4 scenes exercise the closest-hit shadow path (a transparent material exists) and
    chains deeper than 2; the golden comparison above covers bytes, this checks counts against
    the oracle on a different view size and pixel factor."""
    path = scene_path("syn:F4", workdir)
    lights = [[0, 0, 4], [-1.0, 2.0, 4]]
    p = R.RenderParams(width=80, height=45, pf=2, max_lvl=8, lights=lights)
    with R.Scene.load(path, device=0) as sc:
        u8, f32, counts = sc.render(p, want_f32=True)
    of32, ou8, oc = O.OracleScene(path).render(O.make_params(80, 45, 2, 8, lights=lights), nthreads=16)
    assert [int(c) for c in counts] == [int(c) for c in oc]
    _assert_image_close(u8, f32, ou8, of32)


def _query_mix(sc, rng, n):
    """Camera rays, random rays through the scene box, secondary-like rays leaving surface points
    (with the reference's 0.01 offset) and grazing rays."""
    e = sc.export()
    V, F = e["vertices"], e["triangles"]
    lo, hi = V.min(0), V.max(0)
    c = R.default_corners(160, 90)
    t = rng.random((n, 2)).astype(np.float32)
    cam_o = (c[0] * (1 - t[:, :1]) + c[6] * t[:, :1])
    cam_d = (c[1] * (1 - t[:, 1:]) + c[7] * t[:, 1:])
    rnd_o = lo + (hi - lo) * rng.random((n, 3)) * 1.4 - 0.2 * (hi - lo)
    rnd_d = lo + (hi - lo) * rng.random((n, 3))
    k = rng.integers(0, len(F), n)
    bary = rng.random((n, 2))
    bary[bary.sum(1) > 1] = 1 - bary[bary.sum(1) > 1]
    P = V[F[k, 0]] + bary[:, :1] * (V[F[k, 1]] - V[F[k, 0]]) + bary[:, 1:] * (V[F[k, 2]] - V[F[k, 0]])
    dirs = rng.normal(size=(n, 3))
    dirs /= np.linalg.norm(dirs, axis=1)[:, None]
    sec_o = P + 0.01 * dirs
    sec_d = P + dirs
    nrm = e["normals"][k]
    gdir = dirs - (dirs * nrm).sum(1)[:, None] * nrm * (1 - 1e-3)
    gra_o = P - gdir * 0.5
    gra_d = P + gdir * 2.0
    shadow_o = P + 0.1
    shadow_d = np.tile([[0.0, 0.0, 4.0]], (n, 1))
    o = np.concatenate([cam_o, rnd_o, sec_o, gra_o, shadow_o]).astype(np.float32)
    d = np.concatenate([cam_d, rnd_d, sec_d, gra_d, shadow_d]).astype(np.float32)
    return o, d


@pytest.mark.parametrize("width", [2, 4])
@pytest.mark.parametrize("spec", ["ref:dodgeColorTest.obj", "ref:Models/shadow_test.obj", "syn:F4", "syn:C4"])
def test_bvh_matches_brute_force_bitwise(spec, width, workdir, gpu_available):
    path = scene_path(spec, workdir)
    rng = np.random.default_rng(17)
    with R.Scene.load(path, device=0) as sc:
        o, d = _query_mix(sc, rng, 20000)
        sc.set_accel("brute_force")
        bi, bp = sc.intersect_mesh(o, d)
        sc.set_accel("bvh")
        sc.tune("bvh_width", width)
        assert sc.accel() == "bvh"
        vi, vp = sc.intersect_mesh(o, d)
    assert np.array_equal(bi, vi), np.nonzero(bi != vi)[0][:10]
    assert np.array_equal(bp.view(np.uint32), vp.view(np.uint32))
    assert (bi >= 0).sum() > 5000
    # spot-check the brute-force answers against the oracle
    orc = O.OracleScene(path)
    for i in rng.choice(len(o), 150, replace=False):
        oi, opt = orc.intersect_mesh(o[i], d[i])
        assert oi == bi[i] and np.array_equal(opt.view(np.uint32), bp[i].view(np.uint32))


@pytest.mark.parametrize("accel", ["brute_force", "bvh2", "bvh"])
@pytest.mark.parametrize("name", ["F2b_shadow_test_160x120", "F3_spheres_128x72_pf2", "F4_refract_128x72"])
def test_render_accel_modes_match_golden(name, accel, workdir, gpu_available):
    entry = golden_index()[name]
    gu8, gf32 = golden(name)
    with R.Scene.load(scene_path(entry["scene"], workdir), device=0) as sc:
        sc.set_accel("bvh" if accel == "bvh2" else accel)
        sc.tune("bvh_width", 2 if accel == "bvh2" else 4)
        u8, f32, counts = sc.render(_params(entry), want_f32=True)
    assert [int(c) for c in counts] == entry["counts"]
    _assert_image_close(u8, f32, gu8, gf32)


@pytest.mark.parametrize("split", [0, 3, 4, 5])
@pytest.mark.parametrize("chain_from", [0, 1, 2, 255])
@pytest.mark.parametrize("name", ["F2_dodge_200x150", "F2b_shadow_test_160x120", "F3_spheres_128x72_pf2",
                                  "F4_refract_128x72"])
def test_chain_tail_matches_golden(name, chain_from, split, workdir, gpu_available):
    """The per-lane chain launch (RT_TUNE_CHAIN_FROM) from the first step, from the second, and
    never, with grid-stride, dynamic (RT_TUNE_CHAIN_SPLIT 3), dynamic fused-launch wave tasks (4)
    and the per-launch auto choice (5) as query distribution: the golden
    frames and ray counts each time. F4 has transparent materials, so its shadow rays take the
    closest-hit form; dodgeColorTest has always-list triangles."""
    entry = golden_index()[name]
    gu8, gf32 = golden(name)
    with R.Scene.load(scene_path(entry["scene"], workdir), device=0) as sc:
        sc.tune("chain_from", chain_from)
        sc.tune("chain_split", split)
        u8, f32, counts = sc.render(_params(entry), want_f32=True)
    assert [int(c) for c in counts] == entry["counts"]
    _assert_image_close(u8, f32, gu8, gf32)


def test_c4_full_frame_bvh_equals_brute_force(workdir, gpu_available):
    """The benchmark frame itself: BVH and brute-force renders of C4 1920x1080 are byte-identical
    and issue the same queries."""
    p = R.RenderParams(width=1920, height=1080, pf=1, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    with R.Scene.load(scene_path("syn:C4", workdir), device=0) as sc:
        sc.set_accel("bvh")
        a, af, ac = sc.render(p, want_f32=True)
        sc.tune("chain_split", 3)
        a0, af0, ac0 = sc.render(p, want_f32=True)
        sc.tune("chain_split", 0)
        sc.tune("top_nodes", 0)
        a1, af1, ac1 = sc.render(p, want_f32=True)
        sc.tune("top_nodes", 21)
        sc.tune("bvh_width", 2)
        a2, af2, ac2 = sc.render(p, want_f32=True)
        sc.set_accel("brute_force")
        b, bf, bc = sc.render(p, want_f32=True)
    for x, xf, xc in ((a, af, ac), (a0, af0, ac0), (a1, af1, ac1), (a2, af2, ac2)):
        assert [int(v) for v in xc] == [int(v) for v in bc]
        assert np.array_equal(x, b)
        assert np.array_equal(xf.view(np.uint32), bf.view(np.uint32))


@pytest.mark.parametrize("mode,pf,size", [(1, 1, (320, 180)), (1, 2, (200, 110)), (1, 1, (37, 23)), (1, 3, (90, 50))])
def test_batch_order_from_previous_launch_keeps_results(mode, pf, size, workdir, gpu_available):
    """RT_TUNE_BATCH_ORDER: the first render dispatches the chain's batches in screen order and
    times them; the next renders over the same batches dispatch them longest first (pf 3: 63-lane
    batches of 7 pixels). Every render is byte-identical with identical ray counts, with the order
    on or off."""
    p = R.RenderParams(width=size[0], height=size[1], pf=pf, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    with R.Scene.load(scene_path("syn:C4", workdir), device=0) as sc:
        sc.tune("batch_order", 0)
        ref, fref, cref = sc.render(p, want_f32=True)
        sc.tune("batch_order", mode)
        sc.tune("order_every", 2)
        for _ in range(5):
            u8, f32, counts = sc.render(p, want_f32=True)
            assert [int(c) for c in counts] == [int(c) for c in cref]
            assert np.array_equal(u8, ref)
            assert np.array_equal(f32.view(np.uint32), fref.view(np.uint32))


@pytest.mark.parametrize("spec,w,h,pf", [("syn:C4", 320, 180, 1), ("ref:dodgeColorTest.obj", 200, 150, 3),
                                         ("syn:F4", 96, 54, 2), ("syn:F4", 17, 9, 1)])
def test_cold_estimate_order_keeps_results(spec, w, h, pf, workdir, gpu_available):
    """RT_TUNE_COLD_ESTIMATE: a new view's first launch is ordered centre-out (2, k_estimate_center)
    or by the primary-walk estimate (1, k_estimate) + the batch sort, instead of screen order (0);
    later launches by measured durations.
    Every render after RT_TUNE_FORGET_ORDER (cold) and the warm ones after it are byte-identical
    with identical ray counts to screen-order dispatch, with the frame and the shard entry."""
    import torch
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    with R.Scene.load(scene_path(spec, workdir), device=0) as sc:
        sc.tune("batch_order", 0)
        ref, reff, refc = sc.render(p, want_f32=True)
        fb0 = torch.zeros(h * w * 3, dtype=torch.uint8, device="cuda:0")
        sc.render_frame_device(p, 16, 16, fb0.data_ptr(), fb0.numel(), torch.cuda.current_stream().cuda_stream)
        sc.tune("batch_order", 1)
        for est in (2, 1, 0, 2):
            sc.tune("cold_estimate", est)
            sc.tune("forget_order", 1)
            for _ in range(3):
                u8, f32, c = sc.render(p, want_f32=True)
                assert [int(x) for x in c] == [int(x) for x in refc]
                assert np.array_equal(u8, ref) and np.array_equal(f32.view(np.uint32), reff.view(np.uint32))
                fb = torch.full((h * w * 3,), 7, dtype=torch.uint8, device="cuda:0")
                sc.render_frame_device(p, 16, 16, fb.data_ptr(), fb.numel(), torch.cuda.current_stream().cuda_stream)
                assert torch.equal(fb, fb0)


def test_multi_frame_shard_batch_reassembles(workdir, gpu_available):
    """Weak-scaling step shape: a batch of 3 frames of one view, ids g = f*T + t interleaved over 3
    ranks, one rt_render_tiles_device call per rank; every assembled frame equals the render."""
    import torch
    from raytracert_amd import dist
    path = scene_path("syn:F3", workdir)
    p = R.RenderParams(width=100, height=70, pf=1, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    layout = dist.TileLayout(p.width, p.height, 16, 16)
    plan = dist.ShardPlan(layout, 3, frames=3)
    with R.Scene.load(path, device=0) as sc:
        full, _, counts = sc.render(p)
        shards = []
        total = np.zeros(3, np.uint64)
        for rank in range(3):
            buf = torch.zeros(plan.shard_bytes, dtype=torch.uint8, device="cuda:0")
            n, c = sc.render_tiles_device(p, 16, 16, rank, 3, buf.data_ptr(), buf.numel(),
                                          torch.cuda.current_stream().cuda_stream, want_counts=True, frames=3)
            assert n == plan.rank_tiles(rank)
            total += c
            shards.append(buf)
        frames = dist.assemble_plan_torch(torch.cat(shards), plan).cpu().numpy()
    for f in frames:
        assert np.array_equal(f, full)
    assert [int(x) for x in total] == [3 * int(x) for x in counts]


@pytest.mark.parametrize("knobs", [{"xcd_split": 0}, {"xcd_split": 1}, {"xcd_split": 2},
                                   {"xcd_split": 2, "bvh_grid": 3}, {"xcd_split": 1, "bvh_grid": 5},
                                   {"bvh_width": 2, "xcd_split": 2}, {"lds_stack": 1}, {"lds_stack": 5, "bvh_grid": 7},
                                   {"bvh_width": 2, "lds_stack": 2}, {"pipes": 1}, {"pipes": 3},
                                   {"pipes": 4, "xcd_split": 2}, {"shadow_virtual": 0}, {"shadow_virtual": 5},
                                   {"shadow_virtual": 0, "bvh_width": 2}, {"chain_from": 0}, {"chain_from": 1},
                                   {"chain_from": 3}, {"chain_from": 255}, {"chain_from": 0, "lds_stack": 1},
                                   {"chain_from": 1, "bvh_width": 2}, {"chain_from": 0, "pipes": 1},
                                   {"pipes": 2}, {"pipes": 2, "bvh_grid": 4096}, {"bvh_grid": 65536},
                                   {"fuse_pixels": 0}, {"batch_order": 0}, {"batch_order": 0, "chain_split": 3},
                                   {"chain_split": 1}, {"chain_split": 2}, {"chain_split": 3}, {"chain_split": 4},
                                   {"chain_split": 4, "dyn_group": 0}, {"chain_split": 4, "dyn_group": 6},
                                   {"chain_split": 4, "wave_steal": 1}, {"chain_split": 4, "bvh_grid": 3},
                                   {"chain_split": 0}, {"wave_steal": 0},
                                   {"wave_steal": 1}, {"wave_steal": 1, "lds_stack": 1},
                                   {"wave_steal": 1, "bvh_grid": 3}, {"wave_steal": 1, "top_nodes": 0}])
def test_launch_shape_knobs_never_change_results(knobs, workdir, gpu_available):
    """Query distribution (grid-stride, static XCD segments, work-stealing XCD queues), tiny grids
    (fewer blocks than XCDs), tree width and the LDS/HBM split of the traversal stack (1 entry in
    LDS: nearly every push overflows), render pipelines and whether shadow rays come from a
    compacted queue or straight from the hits, and from which step on the chain runs per lane in
    one launch, are placement choices only: byte-identical frames and ray counts."""
    p = R.RenderParams(width=320, height=180, pf=2, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    with R.Scene.load(scene_path("syn:C4", workdir), device=0) as sc:
        ref, reff, refc = sc.render(p, want_f32=True)
        for k, v in knobs.items():
            sc.tune(k, v)
        u8, f32, c = sc.render(p, want_f32=True)
    assert [int(x) for x in c] == [int(x) for x in refc]
    assert np.array_equal(u8, ref) and np.array_equal(f32.view(np.uint32), reff.view(np.uint32))


@pytest.mark.parametrize("spec,w,h,pf,lights", [("ref:dodgeColorTest.obj", 800, 600, 1, 1), ("syn:F4", 160, 90, 2, 2),
                                                ("syn:C4", 480, 270, 1, 2), ("ref:Models/shadow_test.obj", 200, 150, 2, 4)])
def test_wave_steal_matches_plain_walk(spec, w, h, pf, lights, workdir, gpu_available):
    """RT_TUNE_WAVE_STEAL: lanes whose query is done walk subtrees of other lanes' stacks with those
    lanes' rays and fold their finds into the owner's (distance, index) key. The C2 frame (the car's
    slivers and always-list), transparency (closest-hit shadows), pf 2 and up to four lights:
    frames, floats and ray counts equal the plain walk's, and the plain walk equals the oracle on
    sampled pixels elsewhere in the suite."""
    L = [[0, 0, 4], [1.5, 1.5, 4], [-1.5, 1.5, 4], [0, -1.5, 4]][:lights]
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=3 if lights > 1 else 1, lights=L)
    with R.Scene.load(scene_path(spec, workdir), device=0) as sc:
        sc.tune("wave_steal", 0)
        ref, reff, refc = sc.render(p, want_f32=True)
        sc.tune("wave_steal", 1)
        for _ in range(2):
            u8, f32, c = sc.render(p, want_f32=True)
            assert [int(x) for x in c] == [int(x) for x in refc]
            assert np.array_equal(u8, ref) and np.array_equal(f32.view(np.uint32), reff.view(np.uint32))


@pytest.mark.parametrize("spec,w,h,pf,pfy,steal,half,quarter,eighth", [
    ("ref:dodgeColorTest.obj", 400, 300, 1, 1, 1, 512, 8, 0), ("ref:dodgeColorTest.obj", 200, 150, 1, 1, 1, 0, 4096, 0),
    ("syn:C4", 160, 90, 2, 2, 1, 3, 5, 0), ("syn:F4", 96, 54, 4, 4, 1, 0, 2, 8),
    ("syn:C4", 64, 36, 8, 8, 1, 512, 8, 8), ("syn:C4", 80, 45, 4, 8, 1, 512, 8, 8),
    ("syn:F4", 60, 34, 3, 3, 1, 512, 8, 8), ("syn:C4", 72, 40, 2, 8, 1, 8, 8, 8),
    ("ref:dodgeColorTest.obj", 400, 300, 1, 1, 0, 512, 16, 16), ("syn:C4", 333, 187, 3, 3, 0, 100, 50, 20),
    ("syn:C4", 160, 90, 2, 2, 0, 8, 8, 8), ("syn:F4", 60, 34, 3, 3, 0, 0, 0, 4096)])
def test_split_batches_match_plain_walk(spec, w, h, pf, pfy, steal, half, quarter, eighth, workdir, gpu_available):
    """RT_TUNE_STEAL_HALF / _QUARTER / RT_TUNE_SPLIT_EIGHTH: in ordered chain launches (with and
    without stealing) the longest batches run as eight, four or two waves of whole pixels each
    (pf 3: 63-lane batches of 7 pixels split 4+3, 2+2+2+1, 1 x 7); pf 8 x 8 and 4 x 8 (one and two
    pixels per batch) must skip the tiers that would cut a pixel (a half-wave wrote half
    a pixel). Frames, floats and ray counts equal the plain walk's on every launch (the first is
    unordered, later ones ordered, with a part's duration x parts recorded as the batch's cost)."""
    p = R.RenderParams(width=w, height=h, pf=pf, pfy=pfy, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    with R.Scene.load(scene_path(spec, workdir), device=0) as sc:
        sc.tune("wave_steal", 0)
        ref, reff, refc = sc.render(p, want_f32=True)
        sc.tune("wave_steal", steal)
        sc.tune("steal_half", half)
        sc.tune("steal_quarter", quarter)
        sc.tune("split_eighth", eighth)
        for _ in range(4):
            u8, f32, c = sc.render(p, want_f32=True)
            assert [int(x) for x in c] == [int(x) for x in refc]
            assert np.array_equal(u8, ref) and np.array_equal(f32.view(np.uint32), reff.view(np.uint32))


@pytest.mark.parametrize("spec,w,h,pf,lights,half,quarter", [
    ("syn:C4", 160, 90, 1, 2, 0, 4096), ("syn:C4", 240, 135, 1, 2, 512, 64), ("syn:F4", 96, 54, 2, 3, 0, 4096),
    ("ref:dodgeColorTest.obj", 200, 150, 1, 1, 0, 4096), ("syn:C4", 64, 36, 4, 2, 0, 4096), ("syn:F4", 60, 34, 3, 2, 8, 8),
    ("syn:C4", 160, 90, 1, 16, 0, 4096), ("syn:F3", 120, 68, 1, 4, 32, 32)])
def test_quad_walk_matches_plain_walk(spec, w, h, pf, lights, half, quarter, workdir, gpu_available):
    """RT_TUNE_QUAD_WALK: the quarter tier's waves walk with four lanes per ray (a child box per lane,
    DPP ranking, a leaf's triangles side by side, the quad's lexicographic minimum). Opaque (any-hit
    shadows) and transparent (closest-hit shadows, refraction) scenes, the car's always-tested slivers,
    pf 1, 2 and 4 (a quarter is one 16-sample pixel), pf 3 (18-sample quarters: the plain quarter tier),
    1 to 16 lights. Frames, floats and ray counts equal the unsplit plain walk's on every launch."""
    L = [[0, 0, 4], [1.5, 1.5, 4], [-1.5, 1.5, 4], [0, -1.5, 4]] * 4
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=3, lights=L[:lights])
    with R.Scene.load(scene_path(spec, workdir), device=0) as sc:
        sc.tune("wave_steal", 0)
        sc.tune("chain_split", 0)
        sc.tune("steal_half", 0)
        sc.tune("steal_quarter", 0)
        ref, reff, refc = sc.render(p, want_f32=True)
        sc.tune("steal_half", half)
        sc.tune("steal_quarter", quarter)
        sc.tune("quad_walk", 1)
        for i in range(4):
            u8, f32, c = sc.render(p, want_f32=True)
            assert [int(x) for x in c] == [int(x) for x in refc]
            assert np.array_equal(u8, ref) and np.array_equal(f32.view(np.uint32), reff.view(np.uint32)), i


@pytest.mark.parametrize("spec,w,h,pf,lights,half,quarter,eighth", [
    ("syn:C4", 240, 135, 1, 2, 512, 0, 0), ("syn:C4", 240, 135, 1, 4, 64, 64, 64), ("syn:F4", 96, 54, 2, 3, 512, 8, 8),
    ("ref:dodgeColorTest.obj", 200, 150, 1, 1, 512, 0, 0), ("syn:F4", 60, 34, 3, 2, 512, 8, 8),
    ("syn:C4", 160, 90, 1, 16, 32, 32, 32), ("ref:dodgeColorTest.obj", 400, 300, 1, 2, 512, 0, 0),
    ("syn:C4", 480, 270, 1, 2, 4096, 0, 0)])
def test_shadow_helpers_match_plain_walk(spec, w, h, pf, lights, half, quarter, eighth, workdir, gpu_available):
    """RT_TUNE_SHADOW_HELPERS: in split waves (half, quarter, eighth tiers of ordered launches) the
    lanes past a part's samples walk some of their owners' lights; with 1 to 16 lights (1: no helper
    roles), pf 1-3 (pf 3: a 36-lane half leaves no whole helper group), transparency (closest-hit
    shadows, F4). Frames, floats and ray counts equal the unsplit plain walk's on every launch."""
    L = [[0, 0, 4], [1.5, 1.5, 4], [-1.5, 1.5, 4], [0, -1.5, 4]] * 4
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=3, lights=L[:lights])
    with R.Scene.load(scene_path(spec, workdir), device=0) as sc:
        sc.tune("wave_steal", 0)
        sc.tune("chain_split", 0)
        sc.tune("steal_half", 0)
        ref, reff, refc = sc.render(p, want_f32=True)
        sc.tune("steal_half", half)
        sc.tune("steal_quarter", quarter)
        sc.tune("split_eighth", eighth)
        for i in range(5):
            sc.tune("shadow_helpers", 0 if i == 2 else 1)
            u8, f32, c = sc.render(p, want_f32=True)
            assert [int(x) for x in c] == [int(x) for x in refc]
            assert np.array_equal(u8, ref) and np.array_equal(f32.view(np.uint32), reff.view(np.uint32))


@pytest.mark.parametrize("quarter,ncand", [(0, 6), (-1, 9)])
@pytest.mark.parametrize("w,h,pf", [(400, 300, 1), (64, 48, 8), (100, 75, 3)])
def test_wave_steal_auto_trials_keep_results(w, h, pf, quarter, ncand, workdir, gpu_available):
    """RT_TUNE_WAVE_STEAL 2 with RT_TUNE_CHAIN_SPLIT 5 (the defaults) and RT_TUNE_SHADOW_HELPERS 2:
    the first launch over a frame geometry takes its batches dynamically (4), the next re-sort the
    order each time until it was measured under a measured order, then 1 + 2 x candidates launches
    are the timed trials (a warm-up, then two rounds over the candidates: per distribution, plain
    without and with shadow helpers, stealing; with RT_TUNE_STEAL_QUARTER -1, the default, the
    block-dispatch ones also with the quarter tier: nine), later ones use the fastest; every render of
    the sequence equals the plain walk's with block dispatch (pf 8: 64 sub-samples per pixel, where
    the split tiers must stay off), and the trials are reported."""
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=1, lights=[[0, 0, 4], [1.5, 1.5, 4]])
    with R.Scene.load(scene_path("ref:dodgeColorTest.obj", workdir), device=0) as sc:
        sc.tune("wave_steal", 0)
        sc.tune("chain_split", 0)
        sc.tune("steal_quarter", 0)
        ref, reff, refc = sc.render(p, want_f32=True)
        sc.tune("wave_steal", 2)
        sc.tune("chain_split", 5)
        sc.tune("shadow_helpers", 2)
        sc.tune("steal_quarter", quarter)
        sc.tune("forget_order", 1)
        for _ in range(6 + 2 * ncand):
            u8, f32, c = sc.render(p, want_f32=True)
            assert [int(x) for x in c] == [int(x) for x in refc]
            assert np.array_equal(u8, ref) and np.array_equal(f32.view(np.uint32), reff.view(np.uint32))
        t = sc.trials()
        assert t["trials"] == ncand and 0 <= t["choice"] < ncand and len(t["trial_ms"]) == ncand
        assert t["wave_steal"] in (0, 1) and t["chain_split"] in (0, 4) and t["shadow_helpers"] in (0, 1)
        assert t["steal_quarter"] in ((0,) if quarter == 0 else (0, 64))


@pytest.mark.parametrize("spec,w,h,pf,pfy,flags", [("syn:C4", 333, 187, 3, 3, 0), ("syn:F4", 96, 54, 3, 3, 0),
                                                   ("ref:dodgeColorTest.obj", 120, 90, 3, 3, 0), ("syn:F3", 70, 41, 3, 3, 1 << 8),
                                                   ("syn:F4", 17, 9, 5, 5, 0), ("syn:C4", 50, 30, 3, 5, 0),
                                                   ("syn:F4", 40, 22, 7, 9, 0)])
def test_fused_packed_batches_match_frame_pass(spec, w, h, pf, pfy, flags, workdir, gpu_available):
    """Sub-sample counts that do not divide 64 (the reference's default pf 3 x 3 = 9, main.cpp:377-391;
    25, 15 and 63): the fused chain launch packs floor(64 / spp) whole pixels into each wave batch
    (pf 3: 7 pixels x 9 sub-samples in 63 lanes) and sums each pixel's sub-samples by lane shuffles.
    Frames (bytes and floats) and ray counts equal the unfused path's (chain records in HBM, then
    k_frame), with transparency, jittered sampling, batch order and stealing on and off."""
    p = R.RenderParams(width=w, height=h, pf=pf, pfy=pfy, max_lvl=3, lights=[[0, 0, 4], [1.5, 1.5, 4]],
                       flags=R.ALL_FEATURES | flags, seed=7)
    with R.Scene.load(scene_path(spec, workdir), device=0) as sc:
        sc.tune("fuse_pixels", 0)
        ref, reff, refc = sc.render(p, want_f32=True)
        sc.tune("fuse_pixels", 1)
        for steal in (0, 1, 2):
            sc.tune("wave_steal", steal)
            for _ in range(3):   # unordered, then ordered launches
                u8, f32, c = sc.render(p, want_f32=True)
                assert [int(x) for x in c] == [int(x) for x in refc]
                assert np.array_equal(u8, ref) and np.array_equal(f32.view(np.uint32), reff.view(np.uint32))


@pytest.mark.parametrize("spec,w,h,pf", [("ref:dodgeColorTest.obj", 60, 45, 3), ("syn:F4", 48, 27, 3)])
def test_fused_pf3_matches_oracle(spec, w, h, pf, workdir, gpu_available):
    """The reference's default sub-sampling (pixelfactor 3, raytracing.cpp:23) through the fused
    63-lane batches against the oracle at max_lvl 10 (raytracing.cpp:29): same ray counts, the
    golden tests' byte and float bar."""
    path = scene_path(spec, workdir)
    lights = [(0.0, 0.0, 4.0)]
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=10, lights=lights)
    with R.Scene.load(path, device=0) as sc:
        u8, f32, counts = sc.render(p, want_f32=True)
    of32, ou8, ocounts = O.OracleScene(path).render(O.make_params(w, h, pf=pf, max_lvl=10, lights=lights), nthreads=16)
    assert [int(c) for c in counts] == [int(c) for c in ocounts]
    _assert_image_close(u8, f32, ou8, of32)


@pytest.mark.parametrize("spec,w,h,pf", [("syn:F3", 128, 72, 2), ("syn:F4", 96, 54, 2), ("ref:dodgeColorTest.obj", 80, 60, 3)])
def test_stochastic_aa_matches_oracle(spec, w, h, pf, workdir, gpu_available):
    """RT_STOCHASTIC: jittered sub-samples from the counter-based hash of
    include/raytracert.h. The GPU frame matches the oracle's at the same seed (same query counts,
    the golden tests' byte and float bar) and differs from the regular-grid frame."""
    path = scene_path(spec, workdir)
    lights = [(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)]
    p = R.RenderParams(width=w, height=h, pf=pf, max_lvl=3, lights=lights, flags=R.ALL_FEATURES | (1 << 8), seed=0x5EED)
    with R.Scene.load(path, device=0) as sc:
        u8, f32, counts = sc.render(p, want_f32=True)
        g8, _, _ = sc.render(R.RenderParams(width=w, height=h, pf=pf, max_lvl=3, lights=lights), want_f32=False)
    op = O.make_params(w, h, pf=pf, max_lvl=3, lights=lights, flags=O.ALL_FEATURES | O.STOCHASTIC, seed=0x5EED)
    of32, ou8, ocounts = O.OracleScene(path).render(op)
    assert [int(c) for c in counts] == [int(c) for c in ocounts]
    _assert_image_close(u8, f32, ou8, of32)   # the golden-test bar: specular powf may differ by an ulp
    assert not np.array_equal(u8, g8)


@pytest.mark.parametrize("spec", ["syn:F4", "syn:F3", "ref:dodgeColorTest.obj", "ref:Models/shadow_test.obj"])
def test_debug_trace_matches_oracle(spec, workdir, gpu_available):
    """rt_debug_trace (the reference's key 'd', raytracing.cpp:493-510): for
    rays through pixels all over the frame, every trace() call of the chain (ray, hit point,
    triangle, level, per-light shadow outcome) equals the oracle's record bit for bit, the colour
    is within the float tolerance of the oracle's and equals performRayTracing's exactly."""
    path = scene_path(spec, workdir)
    W, H = 96, 64
    lights = [(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)]
    p = R.RenderParams(width=W, height=H, pf=1, max_lvl=6, lights=lights)
    op = O.make_params(W, H, pf=1, max_lvl=6, lights=lights)
    cs = R.default_corners(W, H)
    orc = O.OracleScene(path)
    rng = np.random.default_rng(3)
    chains = 0
    with R.Scene.load(path, device=0) as sc:
        for _ in range(40):
            a, b = rng.random(2).astype(np.float32)
            o = (cs[0] * a + cs[4] * (1 - a)) * b + (cs[2] * a + cs[6] * (1 - a)) * (1 - b)
            d = (cs[1] * a + cs[5] * (1 - a)) * b + (cs[3] * a + cs[7] * (1 - a)) * (1 - b)
            gb, grgb = sc.debug_trace(p, o, d)
            ob, orgb = orc.debug_trace(op, o, d)
            assert len(gb) == len(ob)
            for x, y in zip(gb, ob):
                for k in ("origin", "dest", "hit"):
                    assert np.array_equal(x[k].view(np.uint32), y[k].view(np.uint32)), (k, x, y)
                for k in ("triangle", "level", "shadowed", "lit"):
                    assert x[k] == y[k], (k, x, y)
            assert np.abs(grgb - orgb).max() <= F32_TOL   # specular powf: at most an ulp apart
            prgb, _ = sc.perform_ray_tracing(p, o[None], d[None])
            assert np.array_equal(prgb[0].view(np.uint32), grgb.view(np.uint32))
            chains += len(gb) > 1
    if spec.startswith("syn:"):   # the reference models cover a few percent of the default view
        assert chains > 5


def _sliver_field(path, rng, n=3000):
    """Slivers of 0.8-3 degrees at T0 (the largest acceptance pads the tree uses, and the always-tested
    ones below ~1 degree), a third in exact axis planes, a third tilted by 1e-6..1e-2 rad, a third in
    random orientation, packed into a box so their padded boxes overlap."""
    lines, tris = [], []
    for i in range(n):
        kind = i % 3
        theta = np.deg2rad(rng.uniform(0.8, 3.0))
        L = 10 ** rng.uniform(-2, -0.5)
        base = rng.uniform(-1, 1, 3)
        if kind == 2:
            e1 = rng.normal(size=3); e1 /= np.linalg.norm(e1)
            e2 = rng.normal(size=3); e2 -= (e2 @ e1) * e1; e2 /= np.linalg.norm(e2)
        else:
            ax = i % 3 if kind == 0 else rng.integers(0, 3)
            others = [k for k in range(3) if k != ax]
            phi = rng.uniform(0, 2 * np.pi)
            e1 = np.zeros(3); e2 = np.zeros(3)
            e1[others[0]], e1[others[1]] = np.cos(phi), np.sin(phi)
            e2[others[0]], e2[others[1]] = -np.sin(phi), np.cos(phi)
            if kind == 1:
                e2[ax] = np.sin(10 ** rng.uniform(-6, -2)); e2 /= np.linalg.norm(e2)
        T = np.stack([base, base + L * e1, base + L * rng.uniform(0.3, 1) * (np.cos(theta) * e1 + np.sin(theta) * e2)])
        tris.append(T.astype(np.float32))
    with open(path, "w") as f:
        for T in tris:
            for v in T:
                f.write("v %.9g %.9g %.9g\n" % tuple(v))
        for i in range(n):
            f.write("f %d %d %d\n" % (3 * i + 1, 3 * i + 2, 3 * i + 3))
    return np.array(tris)


@pytest.mark.parametrize("width", [2, 4])
def test_bvh_matches_brute_force_on_sliver_field(width, workdir, gpu_available):
    """The in-plane acceptance pads (r04) where they matter: 3,000 near-threshold slivers, axis-aligned,
    slightly tilted and free, and 120k rays aimed within 1e-4 (barycentric) of their edges and
    vertices from near and far, a third of them grazing. BVH (two- and four-wide) equals brute
    force bit for bit."""
    import os
    rng = np.random.default_rng(41)
    path = os.path.join(workdir, "slivers.obj")
    tris = _sliver_field(path, rng)
    n = 120000
    k = rng.integers(0, len(tris), n)
    T = tris[k].astype(np.float64)
    u, v = T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]
    s = rng.random(n)
    t = rng.random(n) * (1 - s)
    kind = rng.integers(0, 4, n)
    s = np.where(kind == 0, rng.normal(0, 1e-4, n), s)
    t = np.where(kind == 1, rng.normal(0, 1e-4, n), t)
    t = np.where(kind == 2, 1 - s + rng.normal(0, 1e-4, n), t)
    P = T[:, 0] + s[:, None] * u + t[:, None] * v
    d = rng.normal(size=(n, 3)); d /= np.linalg.norm(d, axis=1)[:, None]
    nrm = np.cross(u, v); nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    graze = rng.random(n) < 0.33
    d[graze] -= ((d[graze] * nrm[graze]).sum(1) * (1 - 1e-4 * rng.random(graze.sum())))[:, None] * nrm[graze]
    d /= np.linalg.norm(d, axis=1)[:, None]
    dist = 10 ** rng.uniform(-2, 1, n)
    o = (P - d * dist[:, None]).astype(np.float32)
    dst = (o + d * 10 ** rng.uniform(0, 1.5, n)[:, None]).astype(np.float32)
    with R.Scene.load(path, device=0) as sc:
        info = sc.bvh_info()
        assert info["always"] > 0 and info["leaf_triangles"] > 2000
        sc.set_accel("brute_force")
        bi, bp = sc.intersect_mesh(o, dst)
        sc.set_accel("bvh")
        sc.tune("bvh_width", width)
        vi, vp = sc.intersect_mesh(o, dst)
    assert np.array_equal(bi, vi), np.nonzero(bi != vi)[0][:10]
    assert np.array_equal(bp.view(np.uint32), vp.view(np.uint32))
    assert (bi >= 0).sum() > 30000
