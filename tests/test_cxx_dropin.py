"""include/raytracert_dropin.hpp, the source-level drop-in for the reference's raytracing.h /
mesh.h / Vec3D.h: tests/cxx/dropin_frame.cpp is written against the reference interface (its
globals defined as main.cpp defines them, the 'r' key's loop restated) and compiles with g++
against include/ unchanged. Host mode checks the loader's MyMesh, normals and getMaterial against
the oracle; GPU mode checks that the per-sub-sample performRayTracing loop, the one-call
renderImage and the oracle produce the same image."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from _util import read_ppm, scene_path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dropin_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("dropin") / "dropin_frame")
    lib = os.path.join(ROOT, "raytracert_amd")
    cmd = ["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cxx", "dropin_frame.cpp"), "-L" + lib, "-lrtamd", "-Wl,-rpath," + lib, "-o", out]
    subprocess.run(cmd, check=True)
    return out


def _run(args):
    r = subprocess.run(args, check=True, capture_output=True, text=True, timeout=600)
    out = {}
    for l in r.stdout.splitlines():   # first line of each kind; "material" lines are kept in order
        out.setdefault(l.split()[0], l.split()[1:])
        if l.startswith("material"):
            out.setdefault("materials", []).append(l.split()[1:])
    return out


def _fnv(words):
    h = 1469598103934665603
    for w in words:
        h = ((h ^ int(w)) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return "%016x" % h


def _bits(x):
    return "%08x" % np.float32(x).view(np.uint32)


@pytest.mark.parametrize("spec", ["ref:dodgeColorTest.obj", "ref:cube.obj", "syn:F4"])
def test_dropin_host_mesh_matches_oracle(spec, dropin_bin, workdir):
    path = scene_path(spec, workdir)
    out = _run([dropin_bin, "host", path])
    e = O.OracleScene(path).export()
    V, F, tm, N = e["vertices"], e["triangles"], e["tri_mat"], e["normals"]
    assert out["mesh"][:4] == [str(len(V)), str(len(F)), str(len(F)), str(len(e["materials"]))]
    assert out["mesh"][5] == "1" and out["mesh"][7] == str(len(F))          # light 0, one normal per triangle
    tri_words = np.concatenate([F, tm[:, None]], 1).reshape(-1)
    assert out["digest"] == [_fnv(V.reshape(-1).view(np.uint32)), _fnv(N.reshape(-1).view(np.uint32)), _fnv(tri_words)]
    for line, t in zip(out["materials"], (0, len(F) - 1)):
        m = e["materials"][tm[t]]
        assert line[0] == str(t)
        assert line[1:4] == [_bits(v) for v in m["Kd"]] and line[4] == _bits(m["Ks"][0])
        assert line[5] == _bits(m["Ns"]) and line[6] == _bits(m["Tr"]) and line[7] == str(m["illum"])


@pytest.mark.gpu
@pytest.mark.parametrize("spec,w,h,pf,lvl", [("syn:F4", 40, 24, 2, 3), ("ref:dodgeColorTest.obj", 48, 36, 1, 1)])
def test_dropin_frame_loop_equals_render_and_oracle(spec, w, h, pf, lvl, dropin_bin, workdir, tmp_path, gpu_available):
    path = scene_path(spec, workdir)
    loop_ppm, fast_ppm = str(tmp_path / "loop.ppm"), str(tmp_path / "fast.ppm")
    out = _run([dropin_bin, "gpu", path, str(w), str(h), str(pf), str(lvl), loop_ppm, fast_ppm])
    assert out["frames"][0] == out["frames"][1] == str(w * h * 3)      # loop floats == renderImage floats, bit for bit
    a, b = read_ppm(loop_ppm), read_ppm(fast_ppm)
    assert np.array_equal(a, b)
    lights = [(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)]
    _, ou8, oc = O.OracleScene(path).render(O.make_params(w, h, pf, lvl, lights=lights), nthreads=16)
    d = np.abs(a.astype(np.int16) - ou8.astype(np.int16))
    assert d.max() <= 1 and (d == 0).mean() >= 0.9999
    assert out["frames"][2] == "rays" and out["frames"][3:6] == [str(int(x)) for x in oc]
    c = out["centre"]   # idx, I (3 words), "tri_hit", hit, "same_point", same
    assert c[4] == "tri_hit" and c[6] == "same_point"
    if c[0] != "-1":   # rayIntersectTriangle on intersectMesh's triangle: a hit at the same point
        assert c[5] == "1" and c[7] == "1"
