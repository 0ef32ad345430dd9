"""Mesh API remnants of the reference (VERDICT r03 "What's missing" 4): Mesh::texcoords and
Triangle::t (mesh.cpp:199-209 `vt`, :263-268 the face's texture handles, :290-316 their resize and
fan) through RT_LOAD_TEXCOORDS / rt_scene_texcoords, and Mesh::loadMtl (mesh.cpp:334-460) through
rt_load_mtl. The expectations restate the reference's tokenizer in Python, character by character."""
import gzip
import os

import numpy as np
import pytest

import raytracert_amd as R
from raytracert_amd import _capi

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "models")


def _ref_parse(text):
    """mesh.cpp:95-331 restated for vertices, texcoords and (v, t) triangles."""
    verts, tcs, tris = [], [], []
    for raw in text.splitlines(keepends=True):
        line = raw[:255]
        if not line or line[0] == "#" or line[0].isspace():
            continue
        if line.startswith("v "):
            verts.append([np.float32(x) for x in line.split()[1:4]])
        elif line.startswith("vt "):
            parts = line.split()[1:3]
            t = [np.float32(0), np.float32(0), np.float32(0)]
            for k, x in enumerate(parts):
                try:
                    t[k] = np.float32(x)
                except ValueError:
                    break
            tcs.append(t)
        elif line.startswith("f "):
            s = line[2:] + "\0"
            i = 0
            while s[i] == " ":
                i += 1
            vh, th = [], []
            comp, end = 0, False
            p1 = i
            while p1 is not None:
                p0 = p1
                while s[p1] not in "/\r\n \0":
                    p1 += 1
                if s[p1] != "/":
                    end = True
                tok = s[p0:p1]
                if s[p1] != "\0":
                    p1 += 1
                if s[p1] in "\0\n":
                    p1 = None
                if tok:
                    if comp == 0:
                        vh.append(int(tok) - 1)
                    elif comp == 1:
                        th.append(int(tok) - 1)
                comp += 1
                if end:
                    comp, end = 0, False
            th = (th + [0] * len(vh))[: len(vh)]
            if any(v < 0 for v in vh) or len(vh) < 3:
                continue
            for j in range(len(vh) - 2):
                tris.append(((vh[0], vh[j + 1], vh[j + 2]), (th[0], th[j + 1], th[j + 2])))
    nv = len(verts)
    tris = [t for t in tris if all(v < nv for v in t[0])]   # (the library drops faces past the vertex list)
    tv = np.array([t[0] for t in tris], np.uint32).reshape(-1, 3)
    tt = np.array([[x & 0xFFFFFFFF for x in t[1]] for t in tris], np.uint32).reshape(-1, 3)
    return np.array(verts, np.float32).reshape(-1, 3), np.array(tcs, np.float32).reshape(-1, 3), tv, tt


def _check(path, text):
    sc = R.Scene.load(path, device=R.RT_HOST_ONLY, texcoords=True)
    e = sc.export()
    tc, tt = sc.texcoords()
    v, etc, etv, ett = _ref_parse(text)
    assert np.array_equal(e["vertices"], v)
    assert np.array_equal(e["triangles"], etv)
    assert np.array_equal(tc.view(np.uint32), etc.view(np.uint32))
    assert np.array_equal(tt, ett)
    plain = R.Scene.load(path, device=R.RT_HOST_ONLY).export()   # the fast path's scene is the same
    for k in ("vertices", "triangles", "tri_mat", "normals"):
        assert np.array_equal(plain[k], e[k]), k
    return tc, tt


def test_cube_texcoords_match_reference_parse(tmp_path):
    text = gzip.open(os.path.join(GOLDEN, "cube.obj.gz"), "rt").read()
    p = tmp_path / "cube.obj"
    p.write_text(text)
    tc, tt = _check(str(p), text)
    assert len(tc) == 4 and tt.max() <= 3


def test_texcoord_corner_cases(tmp_path):
    text = "\n".join([
        "v 0 0 0", "v 1 0 0", "v 0 1 0", "v 1 1 0", "v 2 2 0",
        "vt 0.25 0.75", "vt 0.5", "vt 1 2 3", "vt",   # ("vt" alone is not "vt ": no entry)
        "f 1 2 3",                  # no texture handles: resized with 0
        "f 1/1 2/2 4/3 3/4",        # quad: the fan (0, i+1, i+2) for both handles
        "f 1//1 2//2 3//3",         # empty texture component: skipped, then zeros
        "f 1/0 2/1 3/2",            # handle 0 -> -1 as unsigned
        "f 1/1 2/2",                # fewer than 3 vertices: dropped
        "f 1/1 2/2 9/3",            # past the vertex list: dropped with its handles
        "f 5/4 4/3 3/2 2/1 1/1",    # pentagon
        "",
    ])
    p = tmp_path / "t.obj"
    p.write_text(text)
    tc, tt = _check(str(p), text)
    assert len(tc) == 3 and np.array_equal(tc[1], np.float32([0.5, 0, 0])) and np.array_equal(tc[2], np.float32([1, 2, 0]))
    assert tt[0].tolist() == [0, 0, 0] and tt[4].tolist() == [0xFFFFFFFF, 0, 1]


def test_texcoords_need_the_load_flag(tmp_path):
    p = tmp_path / "a.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nvt 1 1\nf 1/1 2/1 3/1\n")
    sc = R.Scene.load(str(p), device=R.RT_HOST_ONLY)
    with pytest.raises(R.RtError):
        sc.texcoords()
    with pytest.raises(R.RtError):   # unknown flag bits
        R.Scene.load(str(p), device=R.RT_HOST_ONLY, threads=0, sequential=True, texcoords=False).texcoords()
    import ctypes as C
    h = C.c_void_p()
    assert _capi.lib().rt_scene_load_obj_ex(str(p).encode(), R.RT_HOST_ONLY, 0x20, C.byref(h)) == _capi.RT_E_ARG


def test_load_mtl_blocks_and_loadmtl_name_filter(tmp_path):
    # dodgeColorTest.mtl: unique names, so the scene's materials after the default are the blocks
    mtl = gzip.open(os.path.join(GOLDEN, "dodgeColorTest.mtl.gz"), "rt").read()
    obj = gzip.open(os.path.join(GOLDEN, "dodgeColorTest.obj.gz"), "rt").read()
    (tmp_path / "dodgeColorTest.mtl").write_text(mtl)
    (tmp_path / "dodgeColorTest.obj").write_text(obj)
    blocks = R.load_mtl(str(tmp_path / "dodgeColorTest.mtl"))
    mats = R.Scene.load(str(tmp_path / "dodgeColorTest.obj"), device=R.RT_HOST_ONLY).export()["materials"]
    assert len(blocks) == len(mats) - 1 and len({n for n, _ in blocks}) == len(blocks)
    for (name, b), m in zip(blocks, mats[1:]):
        assert b == m, name
    # a repeated name and inherited values: every block is returned, loadMtl keeps the first
    (tmp_path / "dup.mtl").write_text("newmtl a\nKd 1 0 0\nNs 10\n\nnewmtl b\nKa 0 1 0\n\nnewmtl a\nKd 0 0 1\n\n"
                                      "newmtl c\nNi 1.5\n\nnewmtl d\nd 0.25\n")
    blocks = R.load_mtl(str(tmp_path / "dup.mtl"))
    assert [n for n, _ in blocks] == ["a", "b", "a", "d"]   # c sets no Kd/Ka/Ks/Tr: never committed
    assert blocks[1][1]["Kd"] == (1.0, 0.0, 0.0) and blocks[1][1]["Ns"] == 10.0   # inherited values
    assert blocks[3][1]["Tr"] == 0.25 and blocks[3][1]["Ni"] == np.float32(1.5)
    (tmp_path / "dup.obj").write_text("mtllib dup.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl a\nf 1 2 3\n")
    mats = R.Scene.load(str(tmp_path / "dup.obj"), device=R.RT_HOST_ONLY).export()["materials"]
    assert len(mats) == 4 and mats[1]["Kd"] == (1.0, 0.0, 0.0)   # default, a (first), b, d
    with pytest.raises(R.RtError):
        R.load_mtl(str(tmp_path / "missing.mtl"))
