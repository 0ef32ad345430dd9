"""Shared helpers for the test suite: fixture inputs and golden outputs."""
from __future__ import annotations

import gzip
import json
import os
import shutil
import sys

import numpy as np

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
GOLDEN = os.path.join(TESTS, "golden")
MODELS = os.path.join(GOLDEN, "models")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

from raytracert_amd import scenes  # noqa: E402


def materialize_models(dst: str) -> str:
    """Decompress the reference's model inputs (CG_Project/*.obj/*.mtl, kept gzip'd as data
    fixtures) into dst, preserving the Models/ sub-directory. Returns dst."""
    for dirpath, _, files in os.walk(MODELS):
        rel = os.path.relpath(dirpath, MODELS)
        out_dir = os.path.join(dst, rel) if rel != "." else dst
        os.makedirs(out_dir, exist_ok=True)
        for f in files:
            if f.endswith(".gz"):
                out = os.path.join(out_dir, f[:-3])
                if not os.path.exists(out):
                    with gzip.open(os.path.join(dirpath, f), "rb") as src, open(out, "wb") as o:
                        shutil.copyfileobj(src, o)
    return dst


def scene_path(spec: str, workdir: str) -> str:
    """spec = 'ref:<file under CG_Project>' or 'syn:<GridSpec name in raytracert_amd.scenes>'."""
    kind, name = spec.split(":", 1)
    if kind == "ref":
        materialize_models(workdir)
        return os.path.join(workdir, name)
    if kind == "syn":
        if name == "balls":     # C3 surrogate (Balls.obj is missing from the reference)
            return scenes.balls_surrogate(workdir)
        return scenes.write_sphere_grid(getattr(scenes, name), workdir, name.lower())
    raise ValueError(spec)


def golden_index() -> dict:
    with open(os.path.join(GOLDEN, "index.json")) as f:
        return json.load(f)


def survey_pins() -> dict:
    with open(os.path.join(GOLDEN, "survey_pins.json")) as f:
        return json.load(f)


def read_ppm(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6" and parts[2] == b"255", "not a P6/255 PPM"
    w, h = (int(v) for v in parts[1].split())
    return np.frombuffer(parts[3], np.uint8).reshape(h, w, 3)


def golden(name: str):
    u8 = read_ppm(os.path.join(GOLDEN, name + ".ppm"))
    f32 = np.load(os.path.join(GOLDEN, name + ".rgb_f32.npy"), allow_pickle=False)
    return u8, f32


def _write_text(d: str, name: str, text: str) -> str:
    with open(os.path.join(d, name), "w", newline="") as f:
        f.write(text)
    return os.path.join(d, name)


def write_adversarial_obj(d: str) -> str:
    """An OBJ (+ two MTLs) of spellings and layouts where a loader could diverge from fgets(256) +
    sscanf("%f") or run out of bounds: lines longer than 255 characters, partial and malformed `v`
    lines, hex/inf/nan/long-digit numbers, usemtl before mtllib and of unknown names, n-gons,
    out-of-range and negative face indices, v/t/n tokens, tabs, CRLF, a NUL byte, no trailing
    newline. Returns the OBJ path (tests/test_loader.py, tests/test_sanitizers.py)."""
    _write_text(d, "a.mtl", "newmtl A\nKd 1 0 0\n\nnewmtl B\nKd 0 1 0\nd 0.5\n\n")
    _write_text(d, "b.mtl", "newmtl C\nKd 0 0 1\n\n")
    rng = np.random.default_rng(7)
    lines = ["# adversarial", "usemtl A", "mtllib a.mtl"]
    spellings = ["1", "-2.5", "+3.25", ".5", "5.", "1e3", "1E-3", "-0.000000", "0.1234567", "123456789.125",
                 "0.12345678901234567890123", "3.4028235e38", "1e39", "1e-40", "1.17549435e-38", "0x1.8p1",
                 "inf", "-infinity", "nan", "1e", "1e+", "1,5", "7abc", "00012.5000", "9999999", "16777217",
                 "1e10", "1e-10", "1e11", "2.5e-11"]
    for i in range(3000):
        r = rng.random()
        if r < 0.55:
            k = rng.integers(0, 4)
            toks = [spellings[rng.integers(0, len(spellings))] if rng.random() < 0.3 else "%.6f" % rng.normal()
                    for _ in range(k)]
            sep = " \t " if rng.random() < 0.1 else " "
            lines.append("v " + sep.join(toks))
        elif r < 0.85:
            n = int(rng.integers(1, 7))
            idx = rng.integers(-2, max(3, len(lines) // 2), n)
            form = rng.integers(0, 3)
            toks = [str(v) if form == 0 else ("%d/%d/%d" % (v, v, v) if form == 1 else "%d//%d" % (v, v)) for v in idx]
            lines.append("f " + " ".join(toks))
        elif r < 0.88:
            lines.append("usemtl " + ["A", "B", "C", "Nope"][rng.integers(0, 4)])
        elif r < 0.89:
            lines.append("mtllib b.mtl" if rng.random() < 0.5 else "mtllib a.mtl")
        elif r < 0.93:   # > 255 characters: later fgets chunks start mid-line
            lines.append("v " + " ".join("%.9f" % x for x in rng.normal(size=int(rng.integers(20, 40)))))
        elif r < 0.95:
            lines.append("f " + " ".join(str(int(x)) for x in rng.integers(1, 50, int(rng.integers(60, 120)))))
        elif r < 0.97:
            lines.append("#" + "x" * int(rng.integers(200, 600)))
        else:
            lines.append(["vt 0 0", "vn 0 0 1", "o thing", "g grp", "s off", "", "   v 1 2 3", "\tf 1 2 3",
                          "v", "f", "vx 1 2 3"][rng.integers(0, 11)])
    text = "\r\n".join(lines[:1500]) + "\r\n" + "\n".join(lines[1500:])
    text = text.replace("v 1 2 3", "v 1\x00 2 3", 1) + "\nv 4 5 6\nf 1 2 3"   # NUL byte, no final newline
    p = _write_text(d, "adv.obj", text)
    return p
