"""The BVH's exactness rests on one claim (raytracert_amd/csrc/bvh.cpp): whenever
rayIntersectTriangle (CG_Project/raytracing.cpp:99-154) accepts a ray, the returned point I lies
inside the triangle's padded acceptance box, widened by the per-ray pad
64*eps*(|o|_1 + M_1). These CPU tests check that claim against the oracle's arithmetic on rays
aimed at the triangle's edges and vertices (where rounding decides), grazing rays, far origins
and badly shaped triangles, and check the built tree's structure on every scene."""
import numpy as np
import pytest

import oracle as O
import raytracert_amd as R
from raytracert_amd.api import bvh_acceptance_box
from _util import scene_path

EPS = 2.0 ** -24


def _rays_near(T, rng, n, far=False):
    """Rays through points around the triangle's boundary (barycentrics within +-1e-3 of the
    edges, some exactly on them), from random origins; a fraction graze the plane."""
    T = np.asarray(T, np.float64)
    u, v = T[1] - T[0], T[2] - T[0]
    nrm = np.cross(u, v)
    nrm /= np.linalg.norm(nrm)
    L = max(np.linalg.norm(u), np.linalg.norm(v))
    s = rng.random(n)
    t = rng.random(n) * (1 - s)
    kind = rng.integers(0, 4, n)
    s = np.where(kind == 0, rng.normal(0, 1e-4, n), s)            # edge s = 0
    t = np.where(kind == 1, rng.normal(0, 1e-4, n), t)            # edge t = 0
    on_hyp = kind == 2                                            # edge s + t = 1
    t = np.where(on_hyp, 1 - s + rng.normal(0, 1e-4, n), t)
    P = T[0] + s[:, None] * u + t[:, None] * v
    dist = L * (1e3 if far else 1.0) * (0.5 + 4 * rng.random(n))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    graze = rng.random(n) < 0.3
    d[graze] -= np.outer(d[graze] @ nrm, nrm)[...] * (1 - 1e-4 * rng.random(graze.sum()))[:, None]
    d /= np.linalg.norm(d, axis=1)[:, None]
    o = P - d * dist[:, None]
    # |dir| of 1-100 scene units, as camera rays (~9) and shadow rays (~4) have: the reference's
    # absolute parallel threshold |n.dir| < 1e-5 (:115) rejects small triangles for short dirs
    dest = o + d * (10 ** rng.uniform(0, 2, n))[:, None]
    return np.stack([o, dest], 1).astype(np.float32)


def _check_triangle(T, rays):
    st, lo, hi = bvh_acceptance_box(T)
    hit, I = O.ray_intersect_triangle_batch(rays, T)
    if st != 0:
        return st, 0
    o = rays[:, 0, :].astype(np.float64)
    m1 = np.abs(np.asarray(T, np.float64)).sum(1).max()
    pad = 64 * EPS * (np.abs(o).sum(1) + m1)
    I = I.astype(np.float64)
    inside = np.all((I >= lo - pad[:, None]) & (I <= hi + pad[:, None]), axis=1)
    bad = hit & ~inside
    assert not bad.any(), (T, rays[bad][:3], I[bad][:3], lo, hi)
    return st, int(hit.sum())


@pytest.mark.parametrize("spec", ["ref:dodgeColorTest.obj", "ref:Models/shadow_test.obj", "syn:C4"])
def test_acceptance_claim_on_scene_triangles(spec, workdir):
    e = R.Scene.load(scene_path(spec, workdir), device=R.RT_HOST_ONLY).export()
    V, F = e["vertices"], e["triangles"]
    rng = np.random.default_rng(11)
    picks = rng.choice(len(F), size=min(len(F), 120), replace=False)
    accepted = 0
    for i in picks:
        T = V[F[i]]
        rays = _rays_near(T, rng, 4000)
        accepted += _check_triangle(T, rays)[1]
    assert accepted > 10000


def test_acceptance_claim_adversarial_triangles():
    rng = np.random.default_rng(5)
    shapes = []
    for _ in range(60):
        base = rng.normal(size=3) * 10 ** rng.uniform(-2, 3)
        scale = 10 ** rng.uniform(-5, 2)
        aspect = 10 ** rng.uniform(0, 3.5)
        a = rng.normal(size=3)
        b = rng.normal(size=3)
        b -= (b @ a) / (a @ a) * a * (1 - 1 / aspect)     # push towards a sliver
        shapes.append(np.stack([base, base + scale * a, base + scale * b]).astype(np.float32))
    statuses = {0: 0, 1: 0, 2: 0}
    accepted = 0
    for T in shapes:
        for far in (False, True):
            st, n = _check_triangle(T, _rays_near(T, rng, 3000, far=far))
            statuses[st] += 1
            accepted += n
    assert statuses[0] > 60 and accepted > 1000


def test_ill_conditioned_and_degenerate_classification():
    # collinear: n == 0 -> never accepted
    st, _, _ = bvh_acceptance_box([[0, 0, 0], [1, 0, 0], [2, 0, 0]])
    assert st == 2
    # extreme sliver (angle ~1e-6 rad at T0): D has almost no correct bits -> always tested
    st, _, _ = bvh_acceptance_box([[0, 0, 0], [1, 0, 0], [1, 1e-6, 0]])
    assert st == 1
    # a plain right triangle gets a tight box
    st, lo, hi = bvh_acceptance_box([[0, 0, 0], [1, 0, 0], [0, 1, 0]])
    assert st == 0 and np.all(lo <= [0, 0, 0]) and np.all(hi >= [1, 1, 0]) and np.all(hi - lo < [1.01, 1.01, 0.01])


@pytest.mark.parametrize("spec", ["ref:cube.obj", "ref:dodgeColorTest.obj", "ref:Models/shadow_test.obj",
                                  "syn:F3", "syn:F4", "syn:C4"])
def test_bvh_structure(spec, workdir):
    s = R.Scene.load(scene_path(spec, workdir), device=R.RT_HOST_ONLY)
    s.bvh_validate()
    info = s.bvh_info()
    nt = s.counts()[1]
    assert info["leaf_triangles"] + info["always"] + info["never"] == nt
    assert 1 <= info["depth"] <= 40
    assert 1 <= info["depth4"] <= info["depth"] and 1 <= info["nodes4"] <= max(info["nodes"], 1)
    if nt > 1000:
        assert info["always"] < nt * 0.005   # dodgeColorTest: 30 slivers with < ~1 degree at T0


def test_bvh_on_tiny_and_degenerate_scenes(tmp_path):
    p = tmp_path / "one.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nv 2 0 0\nf 1 2 3\nf 1 2 4\n")   # second face is degenerate
    s = R.Scene.load(str(p), device=R.RT_HOST_ONLY)
    s.bvh_validate()
    info = s.bvh_info()
    assert info["never"] == 1 and info["leaf_triangles"] == 1


def test_quantised_boxes_on_far_flat_and_tiny_geometry(tmp_path):
    """Four-wide nodes store child boxes as 8-bit offsets on a power-of-two grid; bvh_validate
    decodes every box exactly as the kernel does and checks it contains everything below it. This
    scene mixes coordinates near 1e5 with features of 1e-3, exactly flat clusters (zero extent on
    an axis) and a spread of scales, where the grid is coarsest relative to the children."""
    rng = np.random.default_rng(3)
    lines, nv = [], 0
    for c in range(120):
        base = rng.normal(size=3) * 10 ** rng.uniform(-2, 5)
        scale = 10 ** rng.uniform(-3, 1)
        flat = c % 4 == 0
        for _ in range(6):
            p0 = base + rng.normal(size=3) * scale
            a, b = rng.normal(size=3) * scale, rng.normal(size=3) * scale
            if flat:
                p0[2] = base[2]; a[2] = 0; b[2] = 0
            for v in (p0, p0 + a, p0 + b):
                lines.append("v %.9g %.9g %.9g" % tuple(v))
            lines.append("f %d %d %d" % (nv + 1, nv + 2, nv + 3))
            nv += 3
    p = tmp_path / "far.obj"
    p.write_text("\n".join(lines) + "\n")
    s = R.Scene.load(str(p), device=R.RT_HOST_ONLY)
    s.bvh_validate()
    info = s.bvh_info()
    assert info["nodes4"] >= 1 and info["leaf_triangles"] + info["always"] + info["never"] == 720


def test_parallel_build_is_the_sequential_tree(workdir, monkeypatch):
    """The threaded build (top levels split with parallel scans, subtrees on worker threads) makes
    every node decision the sequential build makes on the same prim range: identical device arrays
    (digest over both trees, the leaf order and the always list)."""
    path = scene_path("syn:C4", workdir)
    digests = {}
    for t in ("1", "3", "8"):
        monkeypatch.setenv("RTAMD_BVH_THREADS", t)
        s = R.Scene.load(path, device=R.RT_HOST_ONLY)
        digests[t] = s.bvh_digest()
        s.bvh_validate()
    assert len(set(digests.values())) == 1, digests


def test_acceptance_claim_on_near_threshold_slivers():
    """Slivers whose angle at T0 puts K eps between 0.02 and 0.2 (the tree's upper limit, ~1 to
    2 degrees): the largest pads the tree uses. Many rays aimed at the edges and vertices, grazing
    and from far away, against the oracle's arithmetic."""
    rng = np.random.default_rng(23)
    n_box = 0
    accepted = 0
    for i in range(40):
        theta = np.deg2rad(rng.uniform(0.95, 2.2))
        L = 10 ** rng.uniform(-2, 2)
        base = rng.normal(size=3) * 10 ** rng.uniform(-1, 2)
        e1 = rng.normal(size=3); e1 /= np.linalg.norm(e1)
        e2 = rng.normal(size=3); e2 -= (e2 @ e1) * e1; e2 /= np.linalg.norm(e2)
        la, lb = L, L * rng.uniform(0.3, 1.0)
        T = np.stack([base, base + la * e1, base + lb * (np.cos(theta) * e1 + np.sin(theta) * e2)]).astype(np.float32)
        for far in (False, True):
            st, n = _check_triangle(T, _rays_near(T, rng, 6000, far=far))
            n_box += st == 0
            accepted += n
    assert n_box >= 60 and accepted > 3000


def test_acceptance_claim_with_in_plane_pads_on_axis_aligned_slivers():
    """The acceptance pad is an in-plane displacement, so the box widens axis k by the pad times
    sqrt(1 - n_k^2) (r04): a triangle in an axis plane gets (almost) no pad along that axis, and
    the off-plane error of I is the per-ray pad's alone. Slivers of 0.95-2.2 degrees (the largest
    pads) in the three axis planes, exactly and tilted by 1e-6 to 1e-2 rad, with rays aimed at
    their edges, grazing and from far away, against the oracle's arithmetic; and the box along
    the normal axis stays far thinner than in the plane."""
    rng = np.random.default_rng(31)
    n_box = accepted = 0
    for i in range(48):
        axis = i % 3
        theta = np.deg2rad(rng.uniform(0.95, 2.2))
        L = 10 ** rng.uniform(-2, 2)
        base = rng.normal(size=3) * 10 ** rng.uniform(-1, 2)
        ax = [k for k in range(3) if k != axis]
        e1 = np.zeros(3); e2 = np.zeros(3)
        phi = rng.uniform(0, 2 * np.pi)
        e1[ax[0]], e1[ax[1]] = np.cos(phi), np.sin(phi)
        e2[ax[0]], e2[ax[1]] = -np.sin(phi), np.cos(phi)
        tilt = 0.0 if i % 2 == 0 else 10 ** rng.uniform(-6, -2)
        e2[axis] = np.sin(tilt); e2 /= np.linalg.norm(e2)
        la, lb = L, L * rng.uniform(0.3, 1.0)
        T = np.stack([base, base + la * e1, base + lb * (np.cos(theta) * e1 + np.sin(theta) * e2)]).astype(np.float32)
        for far in (False, True):
            st, n = _check_triangle(T, _rays_near(T, rng, 6000, far=far))
            n_box += st == 0
            accepted += n
        st, lo, hi = bvh_acceptance_box(T)
        if st == 0 and tilt == 0.0:
            ext = np.asarray(hi, np.float64) - np.asarray(lo, np.float64)
            assert ext[axis] < 1e-3 * ext[ax].max(), (ext, axis)
    assert n_box >= 80 and accepted > 3000


def test_acceptance_claim_on_slivers_up_to_the_tree_limit():
    """Slivers of 0.85-1.05 degree, on both sides of the tree's K eps limit (RT_BVH_MAX_KE 0.2,
    ~1 degree): rays aimed at their edges and vertices, grazing and from far away, against the
    oracle's arithmetic for those that get a box; those above the limit must be classified
    'always tested'."""
    rng = np.random.default_rng(47)
    n_box = n_always = accepted = 0
    for i in range(48):
        theta = np.deg2rad(rng.uniform(0.85, 1.05))
        L = 10 ** rng.uniform(-3, 2)
        base = rng.normal(size=3) * 10 ** rng.uniform(-1, 2)
        e1 = rng.normal(size=3); e1 /= np.linalg.norm(e1)
        e2 = rng.normal(size=3); e2 -= (e2 @ e1) * e1; e2 /= np.linalg.norm(e2)
        la, lb = L, L * rng.uniform(0.3, 1.0)
        T = np.stack([base, base + la * e1, base + lb * (np.cos(theta) * e1 + np.sin(theta) * e2)]).astype(np.float32)
        for far in (False, True):
            st, n = _check_triangle(T, _rays_near(T, rng, 8000, far=far))
            n_box += st == 0
            n_always += st == 1
            accepted += n
    assert n_box >= 10 and n_always >= 10 and accepted > 1000
