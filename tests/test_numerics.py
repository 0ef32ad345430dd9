"""The two glibc behaviours the kernels reproduce without calling libm (refraction(),
CG_Project/raytracing.cpp:296-316), checked against this platform's libm."""
import ctypes as C
import ctypes.util
import os
import re

import numpy as np

LIBM = C.CDLL(ctypes.util.find_library("m"))
LIBM.acosf.argtypes = [C.c_float]
LIBM.acosf.restype = C.c_float
LIBM.powf.argtypes = [C.c_float, C.c_float]
LIBM.powf.restype = C.c_float

THRESH = float(np.frombuffer(np.array([0xBED51136], np.uint32).tobytes(), np.float32)[0])   # -0x1.aa226cp-2
HERE = os.path.dirname(os.path.abspath(__file__))
INC = os.path.join(os.path.dirname(HERE), "raytracert_amd", "build", "powf2_ties.inc")


def f32(bits):
    return np.array([bits], np.uint32).view(np.float32)[0]


def test_acos_threshold():
    """0 < acosf(c) <= 2  <=>  c >= THRESH, for c in [-1, 0): checked on the 20,001 floats around
    the crossing and on 200,000 random negatives (the build-time scan covered all of [-1,0))."""
    assert float(np.float32(THRESH)) == float.fromhex("-0x1.aa226cp-2")
    tb = 0xBED51136
    for b in range(tb - 10000, tb + 10001):
        c = float(f32(b))
        a = LIBM.acosf(c)
        assert (0 < a <= 2) == (c >= THRESH), hex(b)
    rng = np.random.default_rng(0)
    for c in -rng.random(200000).astype(np.float32):
        c = float(c)
        if c == 0.0:
            continue
        a = LIBM.acosf(c)
        assert (0 < a <= 2) == (c >= THRESH)
    assert not (0 < LIBM.acosf(-1.0) <= 2)
    assert np.isnan(LIBM.acosf(-1.5))


def _table():
    txt = open(INC).read()
    body = txt[txt.index("{") + 1: txt.index("}")]
    return np.array([int(x, 16) for x in re.findall(r"0x[0-9a-f]+", body)], np.uint64).astype(np.uint32)


def test_powf2_table_reproduces_glibc():
    t = _table()
    keys = t & 0x7FFFFFFF
    assert np.all(np.diff(keys.astype(np.int64)) > 0)   # sorted, unique
    assert 300000 < len(t) < 500000

    def emulate(x):
        r = np.float32(x) * np.float32(x)
        ax = np.float32(abs(x)).view(np.uint32)
        i = np.searchsorted(keys, ax)
        if ax < 0x40000000 and i < len(keys) and keys[i] == ax:
            rb = np.float32(r).view(np.uint32)
            rb = rb - 1 if (t[i] >> 31) else rb + 1
            r = np.uint32(rb).view(np.float32)
        return np.float32(r)

    rng = np.random.default_rng(1)
    xs = list(f32(k) for k in keys[::97]) + list((rng.random(20000) * 2 - 1).astype(np.float32))
    for x in xs:
        for s in (1, -1):
            xv = np.float32(s * x)
            g = np.float32(LIBM.powf(float(xv), 2.0))
            assert emulate(xv).view(np.uint32) == g.view(np.uint32), (float(xv), g)
