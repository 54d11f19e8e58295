#!/usr/bin/env python3
"""Stand-in scene generators for the benchmark configs.

The reference's own hitchcock.ray / trimesh2.ray lived in ray/assets/, which
is git-ignored (.gitignore:1) and absent; only their renders ship.  These
generators author deterministic stand-ins with the properties the survey
fixes:

  hitchcock.ray   1 unit sphere (diffuse + specular, magenta) + 96 boxes on a
                  log spiral, random axis-angle rotations/scales (seed 378),
                  blue-green colours, a few reflective; 2 cylinders;
                  1 point + 1 directional light; aspect 1.
  trimesh2.ray    procedural architecture (slab, stairs, pillars with
                  gennormals, loungers, a pool surface transmissive with
                  index 1.33, one reflective glass wall, a displaced
                  sculpture), ~60k triangles in <= 20 trimeshes (seed 2);
                  2 point lights + ambient; aspect 16:9 (headline) —
                  trimesh2_square.ray is the same scene at aspect 1,
                  trimesh2_glass.ray the same geometry with reflective /
                  transmissive materials (recursion-heavy config R1).
  dragon.ray      1M-triangle displaced subdivided mesh (seed 7), 2 point
                  lights, aspect 16:9 (generated on demand, not committed).

Usage: python tools/gen_scenes.py [outdir] [--dragon] [--tris N]
"""
import math
import os
import sys

import numpy as np


def fmt(x):
    return repr(float(x))


def v3(a):
    return "(%s, %s, %s)" % (fmt(a[0]), fmt(a[1]), fmt(a[2]))


def hsv(h, s, v):
    i = int(h * 6) % 6
    f = h * 6 - int(h * 6)
    p, q, t = v * (1 - s), v * (1 - f * s), v * (1 - (1 - f) * s)
    return [(v, t, p), (q, v, p), (p, v, t), (p, q, v), (t, p, v), (v, p, q)][i]


def hitchcock(path):
    rng = np.random.default_rng(378)
    out = ["SBT-raytracer 1.0", "",
           "camera {", "  position = (0, 6, 14);", "  viewdir = (0, -0.42, -1);",
           "  updir = (0, 1, 0);", "  fov = 50;", "  aspectratio = 1;", "}", "",
           "point_light {", "  position = (4, 10, 6);", "  color = (1, 1, 1);",
           "  constant_attenuation_coeff = 0.25;", "  linear_attenuation_coeff = 0.003372407;",
           "  quadratic_attenuation_coeff = 0.000045492;", "}", "",
           "directional_light {", "  direction = (-0.3, -1, -0.5);", "  color = (0.45, 0.45, 0.45);", "}", "",
           "ambient_light { color = (0.15, 0.15, 0.15); }", ""]
    # the sphere
    out += ["translate(0, 1.2, 0, scale(1.2, sphere { material = {",
            "  diffuse = (0.7, 0.1, 0.6); specular = (0.8, 0.8, 0.8); shininess = 64;",
            "  reflective = (0.25, 0.25, 0.25); ambient = (0.2, 0.05, 0.2); } }))", ""]
    # floor box
    out += ["translate(0, -0.25, 0, scale(30, 0.5, 30, box { material = {",
            "  diffuse = (0.55, 0.55, 0.5); ambient = (0.3, 0.3, 0.3); specular = (0.1, 0.1, 0.1); shininess = 8; } }))",
            ""]
    for k in range(96):
        a = 0.35 * k
        r = 1.8 * math.exp(0.018 * k) + 0.15 * k
        x, z = r * math.cos(a), r * math.sin(a)
        s = 0.25 + 0.45 * rng.random()
        h = 0.35 + 0.2 * rng.random()
        col = hsv(h, 0.6 + 0.3 * rng.random(), 0.5 + 0.5 * rng.random())
        ax = rng.normal(size=3)
        ax = ax / np.linalg.norm(ax)
        ang = rng.random() * math.pi
        refl = "reflective = (0.4, 0.4, 0.4); " if k % 7 == 0 else ""
        y = s * 0.6 + 0.3 * rng.random()
        out.append("translate(%s, %s, %s, rotate(%s, %s, %s, %s, scale(%s, %s, %s, box { material = { "
                   "diffuse = %s; specular = (0.3, 0.3, 0.3); shininess = 20; %sambient = (0.1, 0.1, 0.1); } })))" % (
                       fmt(x), fmt(y), fmt(z), fmt(ax[0]), fmt(ax[1]), fmt(ax[2]), fmt(ang),
                       fmt(s), fmt(s * (0.6 + 0.8 * rng.random())), fmt(s), v3(col), refl))
    for (x, z, c) in ((-3.5, -2.0, (0.1, 0.6, 0.6)), (3.0, -3.0, (0.2, 0.7, 0.3))):
        out.append("translate(%s, 0, %s, rotate(1, 0, 0, -1.5707963267948966, scale(0.6, 0.6, 2.5, cylinder { "
                   "material = { diffuse = %s; specular = (0.5, 0.5, 0.5); shininess = 40; } })))" % (
                       fmt(x), fmt(z), v3(c)))
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


# ------------------------------------------------------------------ meshes
def mesh_text(verts, faces, material, gennormals=False, indent="  "):
    lines = ["trimesh {", indent + "points = ("]
    lines.append(",\n".join(indent + "  (%s, %s, %s)" % (fmt(v[0]), fmt(v[1]), fmt(v[2])) for v in verts))
    lines.append(indent + ");")
    lines.append(indent + "faces = (")
    lines.append(",\n".join(indent + "  (%d, %d, %d)" % (int(a), int(b), int(c)) for a, b, c in faces))
    lines.append(indent + ");")
    if gennormals:
        lines.append(indent + "gennormals;")
    lines.append(indent + "material = " + material + ";")
    lines.append("}")
    return "\n".join(lines)


def box_mesh(c, s):
    cx, cy, cz = c
    sx, sy, sz = s
    v = []
    for dz in (-1, 1):
        for dy in (-1, 1):
            for dx in (-1, 1):
                v.append((cx + dx * sx / 2, cy + dy * sy / 2, cz + dz * sz / 2))
    f = [(0, 2, 3), (0, 3, 1), (4, 5, 7), (4, 7, 6), (0, 1, 5), (0, 5, 4),
         (2, 6, 7), (2, 7, 3), (0, 4, 6), (0, 6, 2), (1, 3, 7), (1, 7, 5)]
    return v, f


def merge(parts):
    V, Fs = [], []
    for v, f in parts:
        base = len(V)
        V += list(v)
        Fs += [(a + base, b + base, c + base) for a, b, c in f]
    return V, Fs


def cylinder_mesh(c, r, h, nseg, nring, jitter_rng=None):
    v, f = [], []
    for j in range(nring + 1):
        y = c[1] + h * j / nring
        for i in range(nseg):
            a = 2 * math.pi * i / nseg
            rr = r * (1.0 + 0.06 * math.sin(6 * a) * math.sin(math.pi * j / nring))
            v.append((c[0] + rr * math.cos(a), y, c[2] + rr * math.sin(a)))
    for j in range(nring):
        for i in range(nseg):
            a = j * nseg + i
            b = j * nseg + (i + 1) % nseg
            cc = (j + 1) * nseg + i
            d = (j + 1) * nseg + (i + 1) % nseg
            f += [(a, cc, d), (a, d, b)]
    return v, f


def grid_mesh(x0, x1, z0, z1, y, nx, nz, amp, rng, freq=3.0):
    v, f = [], []
    ph = rng.random(4) * 6.28
    for j in range(nz + 1):
        for i in range(nx + 1):
            x = x0 + (x1 - x0) * i / nx
            z = z0 + (z1 - z0) * j / nz
            yy = y + amp * (math.sin(freq * x + ph[0]) * math.cos(freq * 1.3 * z + ph[1]) +
                            0.5 * math.sin(freq * 2.1 * x + 1.7 * z + ph[2]))
            v.append((x, yy, z))
    for j in range(nz):
        for i in range(nx):
            a = j * (nx + 1) + i
            b = a + 1
            c = a + nx + 1
            d = c + 1
            f += [(a, c, d), (a, d, b)]
    return v, f


def sphere_mesh(c, r, nu, nv, amp, rng):
    v, f = [], []
    ph = rng.random(3) * 6.28
    for j in range(nv + 1):
        th = math.pi * j / nv
        for i in range(nu):
            phi = 2 * math.pi * i / nu
            d = 1 + amp * math.sin(5 * phi + ph[0]) * math.sin(4 * th + ph[1])
            v.append((c[0] + r * d * math.sin(th) * math.cos(phi), c[1] + r * d * math.cos(th),
                      c[2] + r * d * math.sin(th) * math.sin(phi)))
    for j in range(nv):
        for i in range(nu):
            a = j * nu + i
            b = j * nu + (i + 1) % nu
            cc = (j + 1) * nu + i
            d = (j + 1) * nu + (i + 1) % nu
            if j > 0:
                f.append((a, b, d) if False else (a, d, b))
            if j < nv - 1:
                f.append((a, cc, d))
    return v, f


def trimesh2(path, aspect, tris_target=60000, glass=False):
    """glass=True: trimesh2_glass.ray, the same geometry with polished,
    reflective and transmissive materials, so the depth-5 ray trees fork
    (RayTracer.cpp:127-165): more reflection / refraction rays than camera
    rays at -r 5 (the recursion-heavy full-frame config)."""
    rng = np.random.default_rng(2)
    scale = tris_target / 60000.0
    meshes = []
    mat_stone = "{ diffuse = (0.62, 0.6, 0.55); ambient = (0.2, 0.2, 0.2); specular = (0.15, 0.15, 0.15); shininess = 12; }"
    mat_wood = "{ diffuse = (0.55, 0.35, 0.2); ambient = (0.15, 0.1, 0.05); specular = (0.3, 0.3, 0.3); shininess = 30; }"
    mat_pillar = "{ diffuse = (0.85, 0.85, 0.8); ambient = (0.25, 0.25, 0.25); specular = (0.6, 0.6, 0.6); shininess = 60; }"
    mat_water = "{ diffuse = (0.05, 0.2, 0.3); specular = (0.8, 0.8, 0.8); shininess = 120; transmissive = (0.75, 0.9, 0.95); reflective = (0.15, 0.15, 0.15); index = 1.33; }"
    mat_glass = "{ diffuse = (0.02, 0.03, 0.04); specular = (0.9, 0.9, 0.9); shininess = 200; reflective = (0.7, 0.75, 0.8); }"
    mat_sculpt = "{ diffuse = (0.7, 0.25, 0.15); ambient = (0.2, 0.08, 0.05); specular = (0.7, 0.6, 0.5); shininess = 80; reflective = (0.2, 0.2, 0.2); }"
    if glass:
        mat_stone = ("{ diffuse = (0.45, 0.44, 0.4); ambient = (0.15, 0.15, 0.15); specular = (0.5, 0.5, 0.5); "
                     "shininess = 90; reflective = (0.35, 0.35, 0.33); }")
        mat_wood = ("{ diffuse = (0.45, 0.28, 0.15); ambient = (0.12, 0.08, 0.04); specular = (0.6, 0.6, 0.6); "
                    "shininess = 70; reflective = (0.25, 0.2, 0.15); }")
        mat_pillar = ("{ diffuse = (0.1, 0.12, 0.12); specular = (0.9, 0.9, 0.9); shininess = 150; "
                      "reflective = (0.3, 0.32, 0.32); transmissive = (0.6, 0.7, 0.7); index = 1.5; }")
        mat_sculpt = ("{ diffuse = (0.08, 0.03, 0.02); specular = (0.9, 0.85, 0.8); shininess = 160; "
                      "reflective = (0.25, 0.2, 0.2); transmissive = (0.7, 0.5, 0.45); index = 1.45; }")
    # slab (terrain-ish floor grid)
    n = max(8, int(60 * math.sqrt(scale)))
    meshes.append((grid_mesh(-14, 14, -18, 6, 0.0, n, n, 0.01, rng), mat_stone, False))
    # stairs
    parts = []
    for k in range(8):
        parts.append(box_mesh((-9.0, 0.15 + 0.3 * k, -6 - 0.6 * k), (5.0, 0.3, 0.6)))
    meshes.append((merge(parts), mat_stone, False))
    # pillars
    nseg = max(8, int(48 * math.sqrt(scale)))
    nring = max(4, int(40 * math.sqrt(scale)))
    for k in range(8):
        x = -8 + 4.5 * (k % 4)
        z = -13.0 if k < 4 else -3.5
        meshes.append((cylinder_mesh((x, 0.0, z), 0.45, 6.0, nseg, nring), mat_pillar, True))
    # pool surface (transmissive water) + pool basin
    nw = max(8, int(70 * math.sqrt(scale)))
    meshes.append((grid_mesh(-2.0, 6.0, -11.0, -5.0, 0.05, nw, nw // 2, 0.03, rng, 4.0), mat_water, True))
    meshes.append((box_mesh((2.0, -0.9, -8.0), (8.2, 1.6, 6.2)), "{ diffuse = (0.1, 0.45, 0.55); ambient = (0.05, 0.15, 0.2); }", False))
    # loungers
    parts = []
    for k in range(4):
        x = -1.5 + 2.2 * k
        parts.append(box_mesh((x, 0.35, -2.8), (0.9, 0.12, 2.2)))
        parts.append(box_mesh((x, 0.7, -3.8), (0.9, 0.8, 0.12)))
        for dx in (-0.4, 0.4):
            for dz in (-0.9, 0.9):
                parts.append(box_mesh((x + dx, 0.15, -2.8 + dz), (0.08, 0.3, 0.08)))
    meshes.append((merge(parts), mat_wood, False))
    # reflective glass wall
    meshes.append((grid_mesh(-14, 14, -17.5, -17.0, 0.0, 4, 1, 0.0, rng), mat_glass, False))
    gw_v, gw_f = [], []
    for (x, y) in ((-12, 0), (12, 0), (12, 7), (-12, 7)):
        gw_v.append((x, y, -16.5))
    gw_f = [(0, 1, 2), (0, 2, 3)]
    meshes[-1] = ((gw_v, gw_f), mat_glass, False)
    # sculpture: displaced sphere
    nu = max(8, int(110 * math.sqrt(scale)))
    meshes.append((sphere_mesh((6.5, 2.0, -9.0), 1.5, nu, nu // 2, 0.12, rng), mat_sculpt, True))
    ntri = sum(len(m[0][1]) for m in meshes)
    out = ["SBT-raytracer 1.0", "", "// trimesh2 stand-in (tools/gen_scenes.py, seed 2), %d triangles in %d trimeshes" % (ntri, len(meshes)),
           "camera {", "  position = (1.0, 3.4, 7.5);", "  viewdir = (0.0, -0.3, -1.0);", "  updir = (0, 1, 0);",
           "  fov = 55;", "  aspectratio = %s;" % fmt(aspect), "}", "",
           "point_light { position = (-4, 9, 2); color = (0.9, 0.85, 0.8);",
           "  constant_attenuation_coeff = 0.2; linear_attenuation_coeff = 0.02; quadratic_attenuation_coeff = 0.002; }",
           "point_light { position = (7, 6, -4); color = (0.5, 0.55, 0.7);",
           "  constant_attenuation_coeff = 0.3; linear_attenuation_coeff = 0.03; quadratic_attenuation_coeff = 0.004; }",
           "ambient_light { color = (0.12, 0.12, 0.14); }", ""]
    for (v, f), mat, gn in meshes:
        out.append(mesh_text(v, f, mat, gn))
        out.append("")
    with open(path, "w") as fh:
        fh.write("\n".join(out) + "\n")
    return ntri


def dragon(path, ntris=1000000):
    """1M-triangle displaced subdivided sphere-ish blob (seed 7)."""
    rng = np.random.default_rng(7)
    nu = int(math.sqrt(ntris))
    nv = ntris // (2 * nu) + 1
    th = np.pi * np.arange(nv + 1) / nv
    ph = 2 * np.pi * np.arange(nu) / nu
    T, PH = np.meshgrid(th, ph, indexing="ij")
    coef = rng.normal(size=(6,))
    d = (1 + 0.15 * np.sin(5 * PH + coef[0]) * np.sin(4 * T + coef[1]) + 0.05 * np.sin(17 * PH + coef[2]) *
         np.sin(13 * T + coef[3]) + 0.02 * np.sin(41 * PH + coef[4]) * np.cos(37 * T + coef[5]))
    X = 2.5 * d * np.sin(T) * np.cos(PH) * 1.6
    Y = 2.5 * d * np.cos(T) + 2.6
    Z = 2.5 * d * np.sin(T) * np.sin(PH)
    V = np.stack([X, Y, Z], -1).reshape(-1, 3)
    j, i = np.meshgrid(np.arange(nv), np.arange(nu), indexing="ij")
    a = j * nu + i
    b = j * nu + (i + 1) % nu
    c = (j + 1) * nu + i
    dd = (j + 1) * nu + (i + 1) % nu
    F = np.concatenate([np.stack([a, c, dd], -1).reshape(-1, 3), np.stack([a, dd, b], -1).reshape(-1, 3)])
    F = F[:ntris]
    with open(path, "w") as fh:
        fh.write("SBT-raytracer 1.0\n\n// dragon stand-in (tools/gen_scenes.py, seed 7), %d triangles\n" % len(F))
        fh.write("camera { position = (0, 3, 11); viewdir = (0, -0.05, -1); updir = (0, 1, 0); fov = 45;"
                 " aspectratio = 1.7777777777777777; }\n")
        fh.write("point_light { position = (-6, 8, 8); color = (1, 0.95, 0.9); constant_attenuation_coeff = 0.2;"
                 " linear_attenuation_coeff = 0.01; quadratic_attenuation_coeff = 0.001; }\n")
        fh.write("point_light { position = (7, 4, 5); color = (0.4, 0.45, 0.6); constant_attenuation_coeff = 0.3;"
                 " linear_attenuation_coeff = 0.02; quadratic_attenuation_coeff = 0.002; }\n")
        fh.write("ambient_light { color = (0.1, 0.1, 0.1); }\n")
        fh.write("translate(0, -0.5, 0, scale(40, 1, 40, box { material = { diffuse = (0.5, 0.5, 0.5);"
                 " ambient = (0.2, 0.2, 0.2); } }))\n")
        fh.write("trimesh {\n  points = (\n")
        fh.write(",\n".join("(%r, %r, %r)" % (float(x), float(y), float(z)) for x, y, z in V))
        fh.write(");\n  faces = (\n")
        fh.write(",\n".join("(%d, %d, %d)" % (p, q, r) for p, q, r in F))
        fh.write(");\n  gennormals;\n  material = { diffuse = (0.3, 0.6, 0.35); ambient = (0.1, 0.2, 0.1);"
                 " specular = (0.6, 0.6, 0.6); shininess = 50; };\n}\n")
    return len(F)


def main():
    outdir = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scenes")
    os.makedirs(outdir, exist_ok=True)
    tris = 60000
    if "--tris" in sys.argv:
        tris = int(sys.argv[sys.argv.index("--tris") + 1])
    hitchcock(os.path.join(outdir, "hitchcock.ray"))
    n = trimesh2(os.path.join(outdir, "trimesh2.ray"), 1.7777777777777777, tris)
    trimesh2(os.path.join(outdir, "trimesh2_square.ray"), 1.0, tris)
    trimesh2(os.path.join(outdir, "trimesh2_glass.ray"), 1.7777777777777777, tris, glass=True)
    print("trimesh2 triangles:", n)
    if "--dragon" in sys.argv:
        print("dragon triangles:", dragon(os.path.join(outdir, "dragon.ray")))


if __name__ == "__main__":
    main()
