"""include/raytracert.hpp, the C++ layer with the reference tracer's names (raytracing.h:8-41):
a g++-built program drives it as the reference's main.cpp would, and its output is checked
against the Python binding and the oracle."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
import raytracert_amd as R
from _util import scene_path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def cxx_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cxx") / "raytracer_api")
    lib = os.path.join(ROOT, "raytracert_amd")
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cxx", "raytracer_api.cpp"), "-L" + lib, "-lrtamd", "-Wl,-rpath," + lib, "-o", out]
    subprocess.run(cmd, check=True)
    return out


def _run(args):
    r = subprocess.run(args, check=True, capture_output=True, text=True, timeout=600)
    return [l.split() for l in r.stdout.splitlines()]


def _bits(x):
    return "%08x" % np.float32(x).view(np.uint32)


def test_cxx_host_layer(cxx_bin, workdir):
    path = scene_path("ref:dodgeColorTest.obj", workdir)
    lines = _run([cxx_bin, "host", path])
    assert lines[0] == ["error_path", str(-1)]                       # RT_E_IO from a missing OBJ
    assert lines[1][:2] == ["lights", "1"] and lines[1][2:] == ["0", "0", "4"]   # light 0 = camera (init)
    mats = R.Scene.load(path, device=R.RT_HOST_ONLY).export()
    tm = mats["tri_mat"]
    for l in lines[2:4]:
        t = int(l[1])
        m = mats["materials"][tm[t]]
        assert l[3:6] == [_bits(v) for v in m["Kd"]] and l[7] == _bits(m["Ks"][0])
        assert l[9] == _bits(m["Ns"]) and l[11] == _bits(m["Tr"]) and int(l[13]) == m["illum"]


@pytest.mark.gpu
def test_cxx_gpu_layer(cxx_bin, workdir, tmp_path, gpu_available):
    path = scene_path("syn:F4", workdir)
    ppm = str(tmp_path / "cxx.ppm")
    lines = _run([cxx_bin, "gpu", path, ppm])
    byk = {}
    for l in lines:
        byk.setdefault(l[0], []).append(l)
    lights = [(0.0, 0.0, 4.0), (1.5, 1.5, 4.0)]
    p = R.RenderParams(width=96, height=64, pf=1, max_lvl=3, lights=lights)
    with R.Scene.load(path, device=0) as sc:
        u8, _, counts = sc.render(p)
        with open(ppm, "rb") as f:
            data = f.read()
        assert data.startswith(b"P6\n96 64\n255\n") and data[len(b"P6\n96 64\n255\n"):] == u8.tobytes()
        assert [int(x) for x in byk["rays"][0][1:]] == [int(c) for c in counts]
        orc = O.OracleScene(path)
        p0 = R.RenderParams(width=96, height=64, pf=1, max_lvl=0, lights=lights)
        for l in byk["ray"]:
            f = lambda a: np.array([int(x, 16) for x in a], np.uint32).view(np.float32)
            o, d, rgb, local = f(l[3:6]), f(l[7:10]), f(l[11:14]), f(l[17:20])
            prgb, _ = sc.perform_ray_tracing(p, o[None], d[None])
            assert np.array_equal(prgb[0].view(np.uint32), rgb.view(np.uint32))
            assert l[15] == "1" and l[-1] == "1"                        # single == batched == debugTrace colour
            lrgb, _ = sc.perform_ray_tracing(p0, o[None], d[None])       # trace(o, d, max_lvl): local shading only
            assert np.array_equal(lrgb[0].view(np.uint32), local.view(np.uint32))
            oi, opt = orc.intersect_mesh(o, d)
            assert int(l[21]) == oi and [int(x, 16) for x in l[23:26]] == list(opt.view(np.uint32))
