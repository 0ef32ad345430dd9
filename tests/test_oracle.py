"""The CPU restatement (oracle/) against the reference's own recorded outputs and hand-derived
known-answer tests. These pin the oracle before it is trusted as the GPU's checker."""
import numpy as np
import pytest

import oracle as O
from _util import scene_path, survey_pins


def test_default_corners_match_reference_run():
    pins = survey_pins()["corners_1920x1080"]
    c = O.default_corners(1920, 1080)
    np.testing.assert_allclose(c[0], pins["o00"], rtol=0, atol=5e-7)
    np.testing.assert_allclose(c[7], pins["d11"], rtol=0, atol=5e-7)
    # origins on the near plane z=3, destinations on the far plane z=-6
    assert np.all(c[0::2, 2] == 3.0) and np.all(c[1::2, 2] == -6.0)


def test_c1_cube_all_black_and_ray_count(workdir):
    pin = survey_pins()["C1"]
    sc = O.OracleScene(scene_path("ref:cube.obj", workdir))
    p = O.make_params(pin["width"], pin["height"], pin["pf"], pin["max_lvl"], lights=pin["lights"])
    f32, u8, counts = sc.render(p)
    assert int(counts.sum()) == pin["rays_total"]
    assert u8.max() == 0 and f32.max() == 0.0


def test_c4_sphere_grid_48x27_ray_count(workdir):
    pin = survey_pins()["C4_48x27"]
    sc = O.OracleScene(scene_path("syn:C4", workdir))
    assert sc.counts()[:2] == (pin["n_vertices"], pin["n_triangles"])
    p = O.make_params(pin["width"], pin["height"], pin["pf"], pin["max_lvl"], lights=pin["lights"])
    _, _, counts = sc.render(p)
    assert int(counts.sum()) == pin["rays_total"]


@pytest.mark.slow
def test_c2_dodge_800x600_ray_counts(workdir):
    pin = survey_pins()["C2"]
    sc = O.OracleScene(scene_path("ref:dodgeColorTest.obj", workdir))
    assert sc.counts()[1] == pin["n_triangles"]
    p = O.make_params(pin["width"], pin["height"], pin["pf"], pin["max_lvl"], lights=pin["lights"])
    _, _, counts = sc.render(p, nthreads=8)
    assert [int(c) for c in counts] == [pin["rays_primary"], pin["rays_secondary"], pin["rays_shadow"]]


# ---- rayIntersectTriangle KATs (raytracing.cpp:99-154). Every input and intermediate below is a
# dyadic rational, so each binary32 operation is exact and the expected result follows by hand.
TRI = [[0, 0, 0], [1, 0, 0], [0, 1, 0]]   # u=(1,0,0) v=(0,1,0) n=(0,0,1) uu=vv=1 uv=0 D=-1


@pytest.mark.parametrize("R,T,hit,I", [
    # straight down onto the interior
    ([[0.25, 0.25, 1], [0.25, 0.25, -1]], TRI, True, [0.25, 0.25, 0]),
    # on the edge s=0 (x=0): accepted (tests are s<0 / s>1, inclusive)
    ([[0, 0.5, 1], [0, 0.5, 0]], TRI, True, [0, 0.5, 0]),
    # on the hypotenuse s+t == 1 exactly: accepted
    ([[0.5, 0.5, 2], [0.5, 0.5, 1]], TRI, True, [0.5, 0.5, 0]),
    # vertex (0,0): accepted
    ([[0, 0, 1], [0, 0, 0.5]], TRI, True, [0, 0, 0]),
    # just outside the hypotenuse: s+t = 1 + 2^-10 -> rejected
    ([[0.5, 0.5 + 2**-10, 1], [0.5, 0.5 + 2**-10, 0]], TRI, False, None),
    # behind the origin: r = -1 < 0 -> rejected (half-line, no r>1 test either way)
    ([[0.25, 0.25, -1], [0.25, 0.25, -2]], TRI, False, None),
    # beyond the destination: r = 2 is still a hit (segment test is commented out, :128)
    ([[0.25, 0.25, 2], [0.25, 0.25, 1]], TRI, True, [0.25, 0.25, 0]),
    # parallel: b = n.dir = 0 < 1e-5 -> rejected
    ([[0.25, 0.25, 1], [1.25, 0.25, 1]], TRI, False, None),
    # nearly parallel: |b| = 2^-17 < 1e-5 -> rejected although the plane is crossed
    ([[0.25, 0.25, 2**-18], [1.25, 0.25, -2**-18]], TRI, False, None),
    # |b| = 2^-16 > 1e-5 -> accepted; r = 0.5, I = (0.75, 0.25, 0)
    ([[0.25, 0.25, 2**-17], [1.25, 0.25, -2**-17]], TRI, True, [0.75, 0.25, 0]),
    # degenerate triangle (collinear): n == 0 -> rejected
    ([[0.25, 0, 1], [0.25, 0, -1]], [[0, 0, 0], [1, 0, 0], [2, 0, 0]], False, None),
    # origin on the plane: a = 0, r = 0 -> accepted at the origin itself
    ([[0.25, 0.25, 0], [0.25, 0.25, -1]], TRI, True, [0.25, 0.25, 0]),
    # from below (b > 0) the test is two-sided
    ([[0.125, 0.5, -1], [0.125, 0.5, 1]], TRI, True, [0.125, 0.5, 0]),
])
def test_ray_intersect_triangle_kat(R, T, hit, I):
    got_hit, got_I = O.ray_intersect_triangle(R, T)
    assert got_hit == hit
    if hit:
        assert got_I.tolist() == I


def test_intersect_mesh_tie_keeps_lowest_index(workdir):
    """Duplicate coplanar triangles hit at exactly the same distance: strict '<' (:183) keeps the
    first one; a nearer triangle later in the list wins."""
    import os
    d = os.path.join(workdir, "ties")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "t.obj"), "w") as f:
        f.write("v 0 0 0\nv 1 0 0\nv 0 1 0\nv 0 0 0.5\nv 1 0 0.5\nv 0 1 0.5\n")
        f.write("f 1 2 3\nf 1 2 3\nf 4 5 6\nf 4 5 6\n")
    sc = O.OracleScene(os.path.join(d, "t.obj"))
    idx, I = sc.intersect_mesh([0.25, 0.25, 2], [0.25, 0.25, -2])
    assert idx == 2 and I.tolist() == [0.25, 0.25, 0.5]
    idx, I = sc.intersect_mesh([0.25, 0.25, -2], [0.25, 0.25, 2])
    assert idx == 0 and I.tolist() == [0.25, 0.25, 0.0]
    idx, I = sc.intersect_mesh([5, 5, 1], [5, 5, -1])
    assert idx == -1 and I.tolist() == [0, 0, 0]


def _fmix32(h):
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def test_stochastic_jitter_matches_header_definition(workdir):
    """RT_STOCHASTIC (an extension: the reference has the regular grid only).
    The oracle's jittered sub-sample positions follow the hash the header defines: check them
    by rendering a scene whose colour is a function of the primary ray alone, one sample per
    pixel (pf 1), against numpy's restatement of the jittered primary ray (the oracle's own
    intersect_mesh supplies the hit)."""
    path = scene_path("syn:F3", workdir)
    s = O.OracleScene(path)
    W, H, seed = 24, 16, 0x5EED
    p = O.make_params(W, H, pf=2, max_lvl=0, lights=[(0.0, 0.0, 4.0)], flags=O.ALL_FEATURES | O.STOCHASTIC, seed=seed)
    f_st, u_st, c_st = s.render(p)
    p_grid = O.make_params(W, H, pf=2, max_lvl=0, lights=[(0.0, 0.0, 4.0)], flags=O.ALL_FEATURES)
    f_gr, _, c_gr = s.render(p_grid)
    assert [int(x) for x in c_st] == [int(x) for x in c_gr]     # same number of queries per kind
    assert not np.array_equal(f_st, f_gr)                      # but other sub-sample positions
    again = s.render(p)[0]
    assert np.array_equal(again.view(np.uint32), f_st.view(np.uint32))   # a pure function of params
    p2 = O.make_params(W, H, pf=2, max_lvl=0, lights=[(0.0, 0.0, 4.0)], flags=O.ALL_FEATURES | O.STOCHASTIC, seed=seed + 1)
    assert not np.array_equal(s.render(p2)[0], f_st)           # the seed matters
    # the hash itself, as the header spells it (key of pixel (3, 2), sub-sample (1, 0))
    key = ((2 * W + 3) * 4 + 1 * 2 + 0) & 0xFFFFFFFF
    h1 = _fmix32(key ^ _fmix32(seed))
    h2 = _fmix32((h1 + 0x9E3779B9) & 0xFFFFFFFF)
    jx, jy = np.float32(h1 >> 8) * np.float32(2.0 ** -24), np.float32(h2 >> 8) * np.float32(2.0 ** -24)
    assert 0 <= jx < 1 and 0 <= jy < 1
