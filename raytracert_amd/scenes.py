"""Deterministic synthetic OBJ/MTL scenes for the benchmark configurations.

The reference ships only small models (CG_Project/cube.obj, dodgeColorTest.obj,
Models/shadow_test.obj) and its Balls.obj is missing (.MISSING_LARGE_BLOBS:2), so the large
configurations of BASELINE.json are synthetic. The generator follows SURVEY.md §8d exactly
(C4: 8x8 grid of 40x21 UV spheres + a 2-triangle back plane = 102,402 triangles / 51,332
vertices; C5: 16x16 grid of 64x32 spheres = 1,015,810 triangles / 508,420 vertices). No RNG:
coordinates are written with %.6f, so every run produces byte-identical files, which the
loader (CG_Project/mesh.cpp:95-331 semantics) turns into identical triangle lists.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

SPHERE_MATERIALS = [
    ("Sph0", (0.8, 0.2, 0.2)),
    ("Sph1", (0.2, 0.8, 0.2)),
    ("Sph2", (0.2, 0.2, 0.8)),
]


@dataclass(frozen=True)
class GridSpec:
    grid: int          # G: spheres per side
    slices: int        # SL
    stacks: int        # ST
    spacing: float     # centre pitch (0.4 for C4, 0.2 for C5)
    radius: float      # 0.1344 for C4, 0.0672 for C5
    back_kd: float = 0.3
    transparent: bool = False   # F4: one sphere material gets d 0.5, Ni 1.5 (refraction path)

    @property
    def n_triangles(self) -> int:
        per = 2 * self.slices + 2 * self.slices * (self.stacks - 2)
        return self.grid * self.grid * per + 2

    @property
    def n_vertices(self) -> int:
        per = 2 + self.slices * (self.stacks - 1)
        return self.grid * self.grid * per + 4


C4 = GridSpec(grid=8, slices=40, stacks=21, spacing=0.4, radius=0.1344)
C5 = GridSpec(grid=16, slices=64, stacks=32, spacing=0.2, radius=0.0672)
# F3/F4 fixtures: small 2x2 grid of 16x9 spheres.
F3 = GridSpec(grid=2, slices=16, stacks=9, spacing=0.4, radius=0.1344)
F4 = GridSpec(grid=2, slices=16, stacks=9, spacing=0.4, radius=0.1344, transparent=True)


def _mtl_text(spec: GridSpec) -> str:
    out = ["# synthetic sphere-grid materials (raytracert_amd.scenes)", ""]
    for i, (name, kd) in enumerate(SPHERE_MATERIALS):
        out.append(f"newmtl {name}")
        out.append("Ns 96.078431")
        out.append("Ka 0.000000 0.000000 0.000000")
        out.append("Kd %.6f %.6f %.6f" % kd)
        out.append("Ks 0.500000 0.500000 0.500000")
        if spec.transparent and i == 2:
            out.append("Ni 1.500000")
            out.append("d 0.500000")
        else:
            out.append("Ni 1.000000")
            out.append("d 1.000000")
        out.append("illum 2")
        out.append("")
    out.append("newmtl Back")
    out.append("Ns 96.078431")
    out.append("Ka 0.000000 0.000000 0.000000")
    out.append("Kd %.6f %.6f %.6f" % (spec.back_kd, spec.back_kd, spec.back_kd))
    out.append("Ks 0.200000 0.200000 0.200000")
    out.append("Ni 1.000000")
    out.append("d 1.000000")
    out.append("illum 2")
    out.append("")
    return "\n".join(out) + "\n"


def _obj_lines(spec: GridSpec, mtl_name: str):
    G, SL, ST, r = spec.grid, spec.slices, spec.stacks, spec.radius
    yield "# synthetic sphere grid G=%d SL=%d ST=%d (raytracert_amd.scenes)\n" % (G, SL, ST)
    yield f"mtllib {mtl_name}\n"
    base = 1  # OBJ indices are 1-based
    for gy in range(G):
        for gx in range(G):
            cx = -1.6 + spec.spacing * (gx + 0.5)
            cy = 0.56 * (-1.6 + spec.spacing * (gy + 0.5))
            cz = 0.0
            verts = [(cx, cy + r, cz)]
            for i in range(1, ST):
                th = math.pi * i / ST
                st, ct = math.sin(th), math.cos(th)
                for j in range(SL):
                    ph = 2.0 * math.pi * j / SL
                    verts.append((cx + r * (st * math.cos(ph)), cy + r * ct, cz + r * (st * math.sin(ph))))
            verts.append((cx, cy - r, cz))
            for v in verts:
                yield "v %.6f %.6f %.6f\n" % v
            top = base
            bottom = base + 1 + SL * (ST - 1)

            def ring(i, j):
                return base + 1 + (i - 1) * SL + (j % SL)

            yield "usemtl %s\n" % SPHERE_MATERIALS[(gx + gy) % 3][0]
            for j in range(SL):
                yield "f %d %d %d\n" % (top, ring(1, j + 1), ring(1, j))
            for i in range(1, ST - 1):
                for j in range(SL):
                    a, b, c, d = ring(i, j), ring(i, j + 1), ring(i + 1, j + 1), ring(i + 1, j)
                    yield "f %d %d %d\n" % (a, b, c)
                    yield "f %d %d %d\n" % (a, c, d)
            for j in range(SL):
                yield "f %d %d %d\n" % (ring(ST - 1, j), ring(ST - 1, j + 1), bottom)
            base += len(verts)
    for v in [(-4.0, -2.5, -0.6), (4.0, -2.5, -0.6), (4.0, 2.5, -0.6), (-4.0, 2.5, -0.6)]:
        yield "v %.6f %.6f %.6f\n" % v
    yield "usemtl Back\n"
    yield "f %d %d %d\n" % (base, base + 1, base + 2)
    yield "f %d %d %d\n" % (base, base + 2, base + 3)


def write_sphere_grid(spec: GridSpec, directory: str, stem: str) -> str:
    """Write `<stem>.obj` + `<stem>.mtl` into `directory`; return the OBJ path."""
    os.makedirs(directory, exist_ok=True)
    obj_path = os.path.join(directory, stem + ".obj")
    mtl_name = stem + ".mtl"
    with open(os.path.join(directory, mtl_name), "w", newline="\n") as f:
        f.write(_mtl_text(spec))
    tmp = obj_path + ".tmp"
    with open(tmp, "w", newline="\n") as f:
        buf = []
        for line in _obj_lines(spec, mtl_name):
            buf.append(line)
            if len(buf) >= 65536:
                f.write("".join(buf))
                buf.clear()
        f.write("".join(buf))
    os.replace(tmp, obj_path)
    return obj_path


def balls_surrogate(directory: str, stem: str = "balls_surrogate") -> str:
    """C3 surrogate for the missing Balls.obj: 3 UV spheres (48x24) + a ground
    quad, using the four materials of CG_Project/Balls.mtl (restated values, Balls.mtl:4-38)."""
    os.makedirs(directory, exist_ok=True)
    mats = [
        ("Material.002", (0.002, 1.0, 0.0)),
        ("Material.003", (0.267942, 0.273673, 0.281009)),
        ("Material.004", (0.420025, 0.420025, 0.420025)),
        ("Material.005", (0.110282, 0.273831, 0.067133)),
    ]
    with open(os.path.join(directory, stem + ".mtl"), "w", newline="\n") as f:
        for name, kd in mats:
            f.write(f"newmtl {name}\nNs 96.078431\nKa 0.000000 0.000000 0.000000\n")
            f.write("Kd %.6f %.6f %.6f\n" % kd)
            f.write("Ks 0.500000 0.500000 0.500000\nNi 1.000000\nd 1.000000\nillum 2\n\n")
    SL, ST = 48, 24
    spheres = [((-0.9, -0.2, 0.0), 0.45, 0), ((0.0, 0.1, -0.4), 0.55, 1), ((0.9, -0.25, 0.2), 0.4, 2)]
    lines = [f"mtllib {stem}.mtl\n"]
    base = 1
    for (cx, cy, cz), r, mi in spheres:
        verts = [(cx, cy + r, cz)]
        for i in range(1, ST):
            th = math.pi * i / ST
            for j in range(SL):
                ph = 2.0 * math.pi * j / SL
                verts.append((cx + r * (math.sin(th) * math.cos(ph)), cy + r * math.cos(th), cz + r * (math.sin(th) * math.sin(ph))))
        verts.append((cx, cy - r, cz))
        lines += ["v %.6f %.6f %.6f\n" % v for v in verts]
        lines.append("usemtl %s\n" % mats[mi][0])
        ring = lambda i, j: base + 1 + (i - 1) * SL + (j % SL)  # noqa: E731
        bottom = base + 1 + SL * (ST - 1)
        lines += ["f %d %d %d\n" % (base, ring(1, j + 1), ring(1, j)) for j in range(SL)]
        for i in range(1, ST - 1):
            for j in range(SL):
                a, b, c, d = ring(i, j), ring(i, j + 1), ring(i + 1, j + 1), ring(i + 1, j)
                lines.append("f %d %d %d\n" % (a, b, c))
                lines.append("f %d %d %d\n" % (a, c, d))
        lines += ["f %d %d %d\n" % (ring(ST - 1, j), ring(ST - 1, j + 1), bottom) for j in range(SL)]
        base += len(verts)
    for v in [(-3.0, -0.7, -3.0), (3.0, -0.7, -3.0), (3.0, -0.7, 2.0), (-3.0, -0.7, 2.0)]:
        lines.append("v %.6f %.6f %.6f\n" % v)
    lines.append("usemtl Material.003\n")
    lines.append("f %d %d %d %d\n" % (base, base + 3, base + 2, base + 1))
    path = os.path.join(directory, stem + ".obj")
    with open(path, "w", newline="\n") as f:
        f.write("".join(lines))
    return path


def orbit_corners(width: int, height: int, frame: int, step_deg: float = 0.25):
    """Corner rays of view `frame` of an orbit: the reference's trackball (traqueboule.h:103-165) turned
    by frame * step_deg degrees about the world y axis. main.cpp sets the modelview to T(0,0,-4) times
    the trackball's rotation R (main.cpp:216-220), so produceRay's unprojected points (main.cpp:300-325)
    are R^-1 applied to the default view's, about the world origin; MyCameraPosition stays the one
    main.cpp:222 computed at start. Returns the 8 x 3 float32 corners (origin00, dest00, ..., dest11)."""
    import numpy as np
    from .api import default_corners
    c = default_corners(width, height).astype(np.float64)
    a = -np.deg2rad(frame * step_deg)
    rot = np.array([[np.cos(a), 0.0, np.sin(a)], [0.0, 1.0, 0.0], [-np.sin(a), 0.0, np.cos(a)]])
    return (c @ rot.T).astype(np.float32)
