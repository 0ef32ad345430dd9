"""GPU parity of single reference functions through the C-ABI:

* rt_ray_intersect_triangle, rayIntersectTriangle (raytracing.cpp:99-154) for independent (ray,
  triangle) pairs: the hand-derived KATs of tests/test_oracle.py, then 40k random and adversarial
  pairs (rays aimed at edges and vertices, near-parallel rays, degenerate and sliver triangles,
  coordinates large enough to overflow) against the oracle, hit flag and point bits.
* calculateNormals (raytracing.cpp:78-86) on the device: a device scene's normals (computed by
  k_face_normals at upload, the ones the renderer reads) equal the host loader's and the oracle's
  bit for bit, degenerate triangles included.
"""
import numpy as np
import pytest

import oracle as O
import raytracert_amd as R
from _util import scene_path

pytestmark = pytest.mark.gpu

from test_oracle import TRI  # noqa: E402  (the dyadic KAT triangle)


def _same_bits(a, b):
    """Bitwise equality, any NaN equal to any NaN (x86 and gfx950 produce different default NaNs)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    both_nan = np.isnan(a) & np.isnan(b)
    return bool(np.all(both_nan | (a.view(np.uint32) == b.view(np.uint32))))


def _pairs(rng, n):
    T = rng.normal(size=(n, 3, 3)).astype(np.float32)
    k = n // 8
    # slivers and degenerate triangles (collinear, repeated vertex)
    T[:k, 2] = T[:k, 0] + (T[:k, 1] - T[:k, 0]) * rng.uniform(-1, 2, (k, 1)).astype(np.float32)
    T[k:2 * k, 2] += rng.normal(scale=1e-4, size=(k, 3)).astype(np.float32) + (T[k:2 * k, 1] - T[k:2 * k, 2])
    T[2 * k:2 * k + 50, 1] = T[2 * k:2 * k + 50, 0]
    # targets: interior, edges, vertices
    bary = rng.uniform(-0.1, 1.1, (n, 2)).astype(np.float32)
    edge = rng.integers(0, 4, n)
    bary[edge == 1, 0] = 0.0
    bary[edge == 2, 1] = 1.0 - bary[edge == 2, 0]
    P = T[:, 0] + bary[:, :1] * (T[:, 1] - T[:, 0]) + bary[:, 1:] * (T[:, 2] - T[:, 0])
    d = rng.normal(size=(n, 3)).astype(np.float32)
    o = (P - d * rng.uniform(0.5, 3.0, (n, 1))).astype(np.float32)
    dest = (o + d * rng.uniform(0.01, 2.0, (n, 1))).astype(np.float32)
    # near-parallel rays: direction in the plane plus a tiny normal component
    m = 3 * k
    nrm = np.cross(T[m:m + k, 1] - T[m:m + k, 0], T[m:m + k, 2] - T[m:m + k, 0])
    inplane = (T[m:m + k, 1] - T[m:m + k, 0])
    dest[m:m + k] = o[m:m + k] + inplane + nrm * rng.normal(scale=1e-5, size=(k, 1)).astype(np.float32)
    # huge coordinates (overflowing intermediates)
    h = 4 * k
    T[h:h + 100] *= np.float32(3e18)
    o[h:h + 100] *= np.float32(3e18)
    dest[h:h + 100] *= np.float32(3e18)
    rays = np.stack([o, dest], 1).astype(np.float32)
    return rays, T


def test_ray_intersect_triangle_kats():
    cases = [
        ([[0.25, 0.25, 1], [0.25, 0.25, -1]], TRI), ([[0, 0.5, 1], [0, 0.5, 0]], TRI),
        ([[0.5, 0.5, 2], [0.5, 0.5, 1]], TRI), ([[0, 0, 1], [0, 0, 0.5]], TRI),
        ([[0.5, 0.5 + 2 ** -10, 1], [0.5, 0.5 + 2 ** -10, 0]], TRI), ([[0.25, 0.25, -1], [0.25, 0.25, -2]], TRI),
        ([[0.25, 0.25, 2], [0.25, 0.25, 1]], TRI), ([[0.25, 0.25, 1], [1.25, 0.25, 1]], TRI),
        ([[0.25, 0.25, 2 ** -18], [1.25, 0.25, -2 ** -18]], TRI), ([[0.25, 0.25, 2 ** -17], [1.25, 0.25, -2 ** -17]], TRI),
        ([[0.25, 0, 1], [0.25, 0, -1]], [[0, 0, 0], [1, 0, 0], [2, 0, 0]]), ([[0.25, 0.25, 0], [0.25, 0.25, -1]], TRI),
        ([[0.125, 0.5, -1], [0.125, 0.5, 1]], TRI),
    ]
    rays = np.array([c[0] for c in cases], np.float32)
    tris = np.array([c[1] for c in cases], np.float32)
    hit, pts = R.ray_intersect_triangle(rays, tris)
    for i, (r, t) in enumerate(cases):
        oh, oi = O.ray_intersect_triangle(r, t)
        assert hit[i] == oh, i
        assert _same_bits(pts[i], oi if oh else np.zeros(3, np.float32)), i
    assert hit.tolist() == [True, True, True, True, False, False, True, False, False, True, False, True, True]


def test_ray_intersect_triangle_random_pairs_match_oracle(gpu_available):
    rng = np.random.default_rng(5)
    rays, tris = _pairs(rng, 40000)
    hit, pts = R.ray_intersect_triangle(rays, tris)
    hits = 0
    for i in range(len(rays)):
        oh, oi = O.ray_intersect_triangle(rays[i], tris[i])
        assert hit[i] == oh, (i, rays[i], tris[i])
        assert _same_bits(pts[i], oi if oh else np.zeros(3, np.float32)), (i, pts[i], oi)
        hits += oh
    assert 5000 < hits < 38000


def test_ray_intersect_triangle_empty_and_errors(gpu_available):
    hit, pts = R.ray_intersect_triangle(np.zeros((0, 2, 3), np.float32), np.zeros((0, 3, 3), np.float32))
    assert hit.shape == (0,) and pts.shape == (0, 3)
    with pytest.raises(R.RtError):
        R.ray_intersect_triangle(np.zeros((1, 2, 3), np.float32), np.zeros((1, 3, 3), np.float32), device=99)


@pytest.mark.parametrize("spec", ["ref:cube.obj", "ref:dodgeColorTest.obj", "ref:Models/shadow_test.obj", "syn:F4",
                                  "syn:C4", "syn:balls"])
def test_device_normals_equal_loader_and_oracle(spec, workdir, gpu_available):
    path = scene_path(spec, workdir)
    with R.Scene.load(path, device=0) as dev, R.Scene.load(path, device=R.RT_HOST_ONLY) as host:
        dn = dev.export()["normals"]
        hn = host.export()["normals"]
    on = O.OracleScene(path).export()["normals"]
    assert dn.shape == on.shape
    assert _same_bits(dn, hn) and _same_bits(dn, on)


def test_device_normals_degenerate_and_extreme_triangles(gpu_available):
    rng = np.random.default_rng(9)
    V = rng.normal(size=(300, 3)).astype(np.float32)
    V[290:] *= np.float32(1e19)          # cross products overflow to inf: normalize gives NaN/0
    V[280:290] *= np.float32(1e-21)      # underflowing edge products: zero-length normals
    F = rng.integers(0, 300, (600, 3)).astype(np.uint32)
    F[:20, 1] = F[:20, 0]                # repeated vertex: n == 0, normalize leaves it
    F[20:40, 2] = F[20:40, 1]
    mats = [dict(Kd=(0.5, 0.5, 0.5), flags=1)]
    with R.Scene.create(V, F, np.zeros(600, np.uint32), mats, device=0) as dev, \
            R.Scene.create(V, F, np.zeros(600, np.uint32), mats, device=R.RT_HOST_ONLY) as host:
        dn = dev.export()["normals"]
        hn = host.export()["normals"]
    assert _same_bits(dn, hn)
    assert np.all(dn[:40] == 0)
