"""include/raytracert_dropin.hpp, the source-level drop-in for the reference's raytracing.h /
mesh.h / Vec3D.h: tests/cxx/dropin_main.cpp is a host written fresh against the reference interface
the way CG_Project/main.cpp uses it (its globals, RGBValue/Image, produceRay, the 'r' loop with one
performRayTracing per sub-sample, keyboard() ending in yourKeyboardFunc, MyMesh.draw() and
yourDebugDraw() from the draw function). It compiles with g++ against include/ only. Host mode checks
the loader's MyMesh, normals and getMaterial against the oracle; GPU mode replays a key session
(feature toggles '1'-'6', pixel factor '+'/'-', 'L' lights, the debugger's '0'/'d'/'c', 'r' frames)
and checks every frame and every 'd' colour against the oracle with the same settings."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from _util import read_ppm, scene_path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F32_TOL = 2e-6


def _build(out, extra):
    lib = os.path.join(ROOT, "raytracert_amd")
    cmd = ["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-Wall", "-Werror"] + extra + [
        os.path.join(ROOT, "tests", "cxx", "dropin_main.cpp"), "-L" + lib, "-lrtamd", "-Wl,-rpath," + lib, "-o", out]
    subprocess.run(cmd, check=True)
    return out


@pytest.fixture(scope="module")
def dropin_bin(tmp_path_factory):
    return _build(str(tmp_path_factory.mktemp("dropin") / "dropin_main"), ["-I" + os.path.join(ROOT, "include")])


def test_dropin_refcompat_headers_compile_unchanged_includes(tmp_path, workdir):
    """The no-edit route: main.cpp's own `#include "raytracing.h"` / `#include "mesh.h"` with
    include/refcompat on the include path (its four headers forward to the drop-in)."""
    exe = _build(str(tmp_path / "dropin_refcompat"), ["-DRTAMD_REFCOMPAT", "-I" + os.path.join(ROOT, "include", "refcompat")])
    lines = _lines([exe, "host", scene_path("ref:cube.obj", workdir)])
    assert lines[0].startswith("mesh 8 12 12 ")


def _lines(args):
    r = subprocess.run(args, check=True, capture_output=True, text=True, timeout=600)
    return r.stdout.splitlines()


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
    lines = _lines([dropin_bin, "host", path])
    out = {}
    for l in lines:
        out.setdefault(l.split()[0], l.split()[1:])
    mats = [l.split()[1:] for l in lines if l.startswith("material")]
    e = O.OracleScene(path).export()
    V, F, tm, N = e["vertices"], e["triangles"], e["tri_mat"], e["normals"]
    assert out["mesh"][:4] == [str(len(V)), str(len(F)), str(len(F)), str(len(e["materials"]))]
    assert out["mesh"][5] == "1" and out["mesh"][7] == str(len(F))          # light 0, one normal per triangle
    tri_words = np.concatenate([F, tm[:, None]], 1).reshape(-1)
    assert out["digest"] == [_fnv(V.reshape(-1).view(np.uint32)), _fnv(N.reshape(-1).view(np.uint32)), _fnv(tri_words)]
    for line, t in zip(mats, (0, len(F) - 1)):
        m = e["materials"][tm[t]]
        assert line[0] == str(t)
        assert line[1:4] == [_bits(v) for v in m["Kd"]] and line[4] == _bits(m["Ks"][0])
        assert line[5] == _bits(m["Ns"]) and line[6] == _bits(m["Tr"]) and line[7] == str(m["illum"])
    # Vec3D.h API: getTwoOrthogonals gives vectors orthogonal to the input; toString's text
    assert abs(float(out["vec"][0])) < 1e-6 and abs(float(out["vec"][1])) < 1e-6
    assert " ".join(out["vec"][2:]) == "(1.000000, 2.000000, 3.000000)"


def _flags(s):
    return sum(1 << i for i, c in enumerate(s) if c == "1")   # Ambient Diffuse Specular Reflection Shadows Refraction


@pytest.mark.gpu
@pytest.mark.parametrize("spec,w,h", [("syn:F4", 40, 24), ("ref:dodgeColorTest.obj", 48, 36)])
def test_dropin_key_session_matches_oracle(spec, w, h, dropin_bin, workdir, tmp_path, gpu_available):
    """A main.cpp-style session through yourKeyboardFunc (raytracing.cpp:453-553): the default
    frame (pf 3, max_lvl 10, light 0 = camera), then ambient off, shadows off, pf 4 and back down to
    2 (clamped at 1 below), a second light ('L'), reflection and refraction off, each rendered by the
    unchanged 'r' loop (one performRayTracing per sub-sample), plus renderImage() once; the debugger
    ('0', 'd' at two mouse positions, 'c'). Every frame equals the oracle's at the settings the
    session printed (same bar as the golden tests), the one-call frame equals the loop's, and each
    'd' prints the oracle's colour of the ray produceRay shot."""
    path = scene_path(spec, workdir)
    prefix = str(tmp_path / "f")
    keys = ["r", "1", "r", "1", "5", "r", "+", "r", "-", "-", "r", "-", "-", "r", "+", "L", "r", "4", "6", "r", "R",
            "0", "d@5,7", "d@20,11", "c", "5", "r"]
    lines = _lines([dropin_bin, "keys", path, str(w), str(h), prefix] + keys)
    frames = [l.split() for l in lines if l.startswith("frame ")]
    assert len(frames) == keys.count("r") + keys.count("R")
    orc = O.OracleScene(path)
    cache = {}
    expect_pf = [3, 3, 3, 4, 2, 1, 2, 2, 2, 2]
    lights_n = [1, 1, 1, 1, 1, 1, 2, 2, 2, 2]
    for i, f in enumerate(frames):
        pfx, pfy = int(f[3]), int(f[4])
        assert pfx == pfy == expect_pf[i]
        if f[5] == "renderImage":
            flags, nl = cache["last"]
        else:
            flags, nl = _flags(f[6]), int(f[8])
            cache["last"] = (flags, nl)
        assert nl == lights_n[i]
        img = read_ppm(f[1])
        key = (pfx, flags, nl)
        if key not in cache:
            lights = [(0.0, 0.0, 4.0)] * nl
            cache[key] = orc.render(O.make_params(w, h, pf=pfx, max_lvl=10, lights=lights, flags=flags), nthreads=16)[1]
        d = np.abs(img.astype(np.int16) - cache[key].astype(np.int16))
        assert d.max() <= 1 and (d == 0).mean() >= 0.9999, (i, f)
    # the one-call frame ('R') is the frame before it, byte for byte
    ri = next(i for i, f in enumerate(frames) if f[5] == "renderImage")
    assert np.array_equal(read_ppm(frames[ri][1]), read_ppm(frames[ri - 1][1]))
    # toggles as the settings printout reports them after the last key
    last = lines[lines.index("------SETTINGS------", len(lines) - 14):]
    assert last[1:7] == ["Ammbient ON", "Diffuse ON", "Specular ON", "Reflection OFF", "Shadow ON", "Refraction OFF"]
    # 'd': the ray produceRay shot and the colour the session printed, against the oracle's trace
    drays = [l.split()[1:] for l in lines if l.startswith("dray ")]
    cols = [l for l in lines if l.startswith("Ray trace color = ")]
    assert len(drays) == len(cols) == 2
    p = O.make_params(w, h, pf=2, max_lvl=10, lights=[(0.0, 0.0, 4.0)] * 2, flags=_flags("111000"))   # shadows off then
    # the recorded (origin, hit) pairs of each 'd' (raytracing.cpp:498-502, then trace()'s :398-401 per call that hit)
    groups, cur = [], None
    for l in lines:
        if l.startswith("dray "):
            cur = []
            groups.append(cur)
        elif l.startswith("dpair "):
            cur.append(np.array([int(x, 16) for x in l.split()[1:]], np.uint32))
    assert len(groups) == 2
    for r, c, pairs in zip(drays, cols, groups):
        v = np.array([int(x, 16) for x in r], np.uint32).view(np.float32)
        recs, rgb = orc.debug_trace(p, v[:3], v[3:])
        got = np.array([float(x) for x in c.split("(")[1].rstrip(")").split(",")], np.float32)
        assert np.abs(got - rgb).max() <= 1e-6 + F32_TOL
        first = recs[0]["hit"] if recs and recs[0]["triangle"] >= 0 else np.zeros(3, np.float32)
        want = [np.concatenate([v[:3], first])] + [np.concatenate([b["origin"], b["hit"]]) for b in recs if b["triangle"] >= 0]
        assert len(pairs) == len(want)
        for a, b in zip(pairs, want):
            assert np.array_equal(a, np.asarray(b, np.float32).view(np.uint32))
    assert "Ray trace history cleared" in lines


@pytest.mark.gpu
def test_dropin_literal_loop_uses_one_gpu_call_per_frame(dropin_bin, workdir, tmp_path, gpu_available):
    """The unchanged 'r' loop at the reference's defaults (500 x 500, pf 3, max_lvl 10: 2.25M
    performRayTracing calls): the drop-in answers the loop's sub-samples from one frame-wide GPU
    trace, so the loop takes well under a second, and its frame equals renderImage()'s."""
    path = scene_path("ref:dodgeColorTest.obj", workdir)
    prefix = str(tmp_path / "g")
    lines = _lines([dropin_bin, "keys", path, "500", "500", prefix, "T", "V:200", "R", "P:300"])
    fr = [l.split() for l in lines if l.startswith("frame ")]
    assert float(fr[0][10]) < 5000.0   # ms: the whole literal loop
    assert np.array_equal(read_ppm(fr[0][1]), read_ppm(fr[1][1]))
    # 200 records of the frame against the per-call path (the loop's own ray, trace() of it): bit for bit
    v = next(l.split() for l in lines if l.startswith("verify "))
    assert v[1] == "200" and v[4] == "0" and v[6] == "0" and v[8] == "0", v
    single = next(l.split() for l in lines if l.startswith("single "))
    assert float(single[4]) > 0


@pytest.mark.gpu
def test_dropin_session_with_more_lights_than_inline(dropin_bin, workdir, tmp_path, gpu_available):
    """'L' appends a light on every press (main.cpp:334-336) and shade() loops over all of them
    (raytracing.cpp:342): 19 presses give 20 lights (more than RT_MAX_LIGHTS, through
    rt_params.light_list), 'r' and renderImage() render them, and 16 more presses (36 lights, the
    per-step kernels) render again. Every frame equals the oracle's."""
    path = scene_path("syn:F4", workdir)
    prefix = str(tmp_path / "m")
    keys = ["-", "-"] + ["L"] * 19 + ["r", "R"] + ["L"] * 16 + ["r"]
    lines = _lines([dropin_bin, "keys", path, "40", "24", prefix] + keys)
    frames = [l.split() for l in lines if l.startswith("frame ")]
    assert len(frames) == 3
    orc = O.OracleScene(path)
    for f, nl in zip(frames, (20, 20, 36)):
        if f[5] != "renderImage":
            assert int(f[8]) == nl
        ou8 = orc.render(O.make_params(40, 24, pf=1, max_lvl=10, lights=[(0.0, 0.0, 4.0)] * nl), nthreads=16)[1]
        d = np.abs(read_ppm(f[1]).astype(np.int16) - ou8.astype(np.int16))
        assert d.max() <= 1 and (d == 0).mean() >= 0.9999, f


def test_dropin_mesh_texcoords_and_loadmtl(dropin_bin, workdir, tmp_path):
    """Mesh::texcoords / Triangle::t as mesh.cpp loads them (cube.obj has `vt` and v/vt/vn faces),
    equal to rt_scene_texcoords; Mesh::loadMtl as a separate call: a repeated name keeps its first
    block, inherited values, the index the reference builds (VERDICT r03 "What's missing" 4)."""
    path = scene_path("ref:cube.obj", workdir)
    (tmp_path / "dup.mtl").write_text("newmtl a\nKd 1 0 0\nNs 10\n\nnewmtl b\nKa 0 1 0\n\nnewmtl a\nKd 0 0 1\n\n"
                                      "newmtl c\nNi 1.5\n\nnewmtl d\nd 0.25\n")
    lines = _lines([dropin_bin, "host", path, str(tmp_path / "dup.mtl")])
    tcl = next(l.split()[1:] for l in lines if l.startswith("texcoords "))
    import raytracert_amd as R
    tc, tt = R.Scene.load(path, device=R.RT_HOST_ONLY, texcoords=True).texcoords()
    assert int(tcl[0]) == len(tc) == 4
    assert tcl[1] == _fnv(tc.reshape(-1).view(np.uint32)) and tcl[2] == _fnv(tt.reshape(-1))
    lm = next(l.split()[1:] for l in lines if l.startswith("loadmtl "))
    assert lm == ["1", "3", "a=0", "b=1", "d=2"]
    mt = [l.split()[1:] for l in lines if l.startswith("mtl ")]
    assert [m[0] for m in mt] == ["a", "b", "d"]
    assert mt[0][1] == _bits(1.0) and mt[1][1] == _bits(1.0) and mt[1][2] == _bits(1.0)   # b inherits a's Kd
    assert mt[2][3] == _bits(0.25) and mt[0][4] == _bits(10.0)
    lines = _lines([dropin_bin, "host", path, str(tmp_path / "missing.mtl")])
    assert next(l for l in lines if l.startswith("loadmtl ")).split()[1:3] == ["0", "0"]


@pytest.mark.gpu
def test_dropin_loop_with_fma_contraction_still_uses_frame_trace(workdir, tmp_path, gpu_available):
    """a host built with GCC's default -ffp-contract=fast on an FMA target makes the 'r'
    loop's rays with FMAs, so they differ from the device's (which follow the reference's x86-64 build,
    no FMA). The drop-in then traces the loop's own rays, made by the header's loop_ray in the host's
    translation unit, in one call: the literal loop still takes well under a second (the per-call path
    would take minutes), its frame records say so, and the frame is the one-call frame's up to the
    few pixels whose rays round differently."""
    exe = _build(str(tmp_path / "dropin_fma"), ["-mfma", "-ffp-contract=fast", "-I" + os.path.join(ROOT, "include")])
    path = scene_path("ref:dodgeColorTest.obj", workdir)
    # (bounded: the per-call path would take ~150 s per frame)
    r = subprocess.run([exe, "keys", path, "500", "500", str(tmp_path / "c"), "T", "T", "V:200", "R"], check=True,
                       capture_output=True, text=True, timeout=120)
    lines = r.stdout.splitlines()
    fr = [l.split() for l in lines if l.startswith("frame ")]
    cache = [(int(l.split()[2]), int(l.split()[4])) for l in lines if l.startswith("cache host_ray_frames")]
    assert float(fr[1][10]) < 5000.0, fr[1]
    assert cache[-1][0] >= 1, "the FMA build's rays matched the device's: this test no longer covers the fallback"
    # the second frame of the same view goes straight to the host's rays (one device frame
    # trace in the session, the first frame's, whose rays turned out not to be the loop's)
    assert cache[0][1] == 1 and cache[1][1] == 1, cache
    loop, one = read_ppm(fr[1][1]), read_ppm(fr[2][1])
    assert (loop == one).mean() >= 0.999
    # the cached colours are trace() of the host's own rays, bit for bit (the per-call path, 200 records)
    v = next(l.split() for l in lines if l.startswith("verify "))
    assert v[1] == "200" and v[4] == "0" and v[6] == "0" and v[8] == "1", v
