"""CPU-side tests (no GPU): the C ABI library and its exports, the .ray
loader's behaviour, BVH structural identity with the restated KdTree,
primitive known-answer tests through the CPU restatement, and the committed
golden fixtures."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, NEWSCENE, ROOT, cli_opts, scene_path

KAT = os.path.join(GOLDEN, "kat")
PKG_DIR = os.path.join(ROOT, "cs378hgraphics-raytracer_amd")


@pytest.fixture(scope="session", autouse=True)
def built():
    if not all(os.path.exists(os.path.join(PKG_DIR, p)) for p in ("lib/librtx_host.so", "lib/librtx_hip.so",
                                                                    "bin/ray")):
        subprocess.run(["make", "-C", PKG_DIR, "-j8", "all"], check=True, capture_output=True)
    if not os.path.exists(os.path.join(ROOT, "scenes", "trimesh2.ray")):
        subprocess.run(["python3", os.path.join(ROOT, "tools", "gen_scenes.py")], check=True, capture_output=True)


# ------------------------------------------------------------------ C ABI
def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^\s*(?:rtx_status|const char\*|int32_t)\s+(rtx_\w+)\s*\(", txt, re.M)))


def test_hip_library_exports_every_declared_symbol(pkg):
    lib = C.CDLL(os.path.join(PKG_DIR, "lib", "librtx_hip.so"))
    names = _declared("rtx.h")
    assert len(names) >= 7
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(pkg.HIP_SYMBOLS)


def test_host_library_exports_every_declared_symbol(pkg):
    lib = C.CDLL(os.path.join(PKG_DIR, "lib", "librtx_host.so"))
    names = _declared("rtx_host.h")
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(pkg.HOST_SYMBOLS)


def test_struct_sizes_match_header_layout(pkg):
    # sizes fixed by rtx.h (RtxNode 64 B, RtxObject 256 B, RtxFace 96 B, hit record 32 B)
    assert C.sizeof(pkg.RtxHitRecord) == 32
    assert C.sizeof(pkg.RtxRenderParams) == 4 * 10 + 8 * 4 + 4 * 4


def test_shard_pixel_accounting(pkg):
    opts = pkg.RenderOptions.from_cli("-w 100 -r 1".split())
    tot = sum(pkg.shard_pixels(opts, 70, 32, s, 3, True) for s in range(3))
    tiles = ((100 + 31) // 32) * ((70 + 31) // 32)
    assert tot == tiles * 32 * 32
    assert pkg.shard_pixels(opts, 70, 0, 0, 1, False) == 100 * 70


# ------------------------------------------------------------------ loader
def test_fixtures_parse(pkg):
    expect = {  # objects, lights (ray/newScene/*.ray)
        "box_cyl_opaque_shadow_spotlight.ray": (2, 1), "concrete_1.ray": (1, 1), "concrete_2.ray": (1, 3),
        "concrete_3.ray": (1, 3), "distance.ray": (3, 2), "lava_box.ray": (4, 1), "spheres_overlap.ray": (4, 1),
    }
    for name, (no, nl) in expect.items():
        h = pkg.HostScene(os.path.join(NEWSCENE, name))
        assert (h.info.n_objects, h.info.n_lights) == (no, nl), name
    h = pkg.HostScene(os.path.join(NEWSCENE, "concrete_1.ray"))
    assert h.info.n_textures == 1  # lava_bump.bmp


def test_image_height_rule(pkg):
    # CommandLineUI.cpp:156: (int)(w / aspect + 0.5)
    assert pkg.host_lib().rtx_image_height(1920, 1.7777777777777777) == 1080
    assert pkg.host_lib().rtx_image_height(512, 1.0) == 512
    h = pkg.HostScene(scene_path("trimesh2.ray"))
    assert h.height_for(1920) == 1080


@pytest.mark.parametrize("text,needle", [
    ("SBT-raytracer 1.2\n", "too high"),
    ("SBT-raytracer 1.0\ncamera { viewdir = (0,0,-1); }\n", "updir"),
    ("SBT-raytracer 1.0\n{ material = { diffuse = (1,0,0); } sphere {} }\n", "Expected: '}' or geometry"),
    ("SBT-raytracer 1.0\nmaterial = { name = m; diffuse = (1,0,0); }\nsphere { material = m; }\n", "syntax error"),
    ("SBT-raytracer 1.0\ntrimesh { points = ((0,0,0),(1,0,0),(0,1,0)); faces = ((0,1,5)); }\n", "Bad face"),
    ("SBT-raytracer 1.0\nsphere { material = { diffuse = map(\"nope.bmp\"); } }\n", "Unable to load texture"),
    ("SBT-raytracer 1.0\nteapot {}\n", "Expected: geometry"),
    ("SBT-raytracer 1.0\nsphere {} /* unterminated\n", "Unterminated comment"),
    ("SBT-raytracer 1.0\nsphere {} ?\n", "unexpected character"),
])
def test_parser_errors_like_reference(pkg, tmp_path, text, needle):
    p = tmp_path / "bad.ray"
    p.write_text(text)
    with pytest.raises(pkg.RtxError) as e:
        pkg.HostScene(str(p))
    assert needle in str(e.value)


def test_parser_quirks(pkg):
    # polymesh fan triangulation + gennormals + colour alias + summed ambient
    h = pkg.HostScene(os.path.join(KAT, "quad_gennormals.ray"))
    assert h.info.n_faces == 2
    assert abs(h.desc.ambient[0] - 0.2) < 1e-15 and abs(h.desc.ambient[1] - 0.30000000000000004) < 1e-15
    # the degenerate face (0,0,3) is dropped (trimesh.cpp:46-53)
    h = pkg.HostScene(os.path.join(KAT, "triangle.ray"))
    assert h.info.n_faces == 1


def test_bvh_identical_to_restated_kdtree(pkg, orc):
    """The product's flattened BVH (node boxes, split order, leaf items) hashes
    equal the oracle's pointer KdTree (kdTree.h:27-78) on every scene."""
    scenes = [os.path.join(NEWSCENE, n) for n in sorted(os.listdir(NEWSCENE)) if n.endswith(".ray")]
    scenes += [scene_path("hitchcock.ray"), scene_path("trimesh2.ray")]
    for s in scenes:
        h = pkg.HostScene(s)
        a, b = orc.bvh_hash(pkg, s)
        assert (h.info.scene_bvh_hash, h.info.mesh_bvh_hash) == (a, b), s


# ------------------------------------------------------------------ known answers
def _probe(pkg, orc, scene, p, d):
    return orc.probe(pkg, os.path.join(KAT, scene), p, d)


def test_kat_sphere(pkg, orc):
    hit, t, n, obj, face = _probe(pkg, orc, "sphere.ray", (0, 0, 5), (0, 0, -1))
    assert hit and t == 4.0 and n == (0.0, 0.0, 1.0) and obj == 0 and face == -1
    hit, t, n, _, _ = _probe(pkg, orc, "sphere_scaled.ray", (0, 0, 5), (0, 0, -1))
    assert hit and t == 3.0 and n == (0.0, 0.0, 1.0)
    hit, *_ = _probe(pkg, orc, "sphere.ray", (0, 2, 5), (0, 0, -1))
    assert not hit


def test_kat_box_and_slab_quirk(pkg, orc):
    hit, t, n, _, _ = _probe(pkg, orc, "box.ray", (0, 0, 5), (0, 0, -1))
    assert hit and t == 4.5 and n == (0.0, 0.0, 1.0)
    # on the face boundary x = 0.5: inclusive test => hit (Box.cpp:36)
    hit, t, _, _, _ = _probe(pkg, orc, "box.ray", (0.5, 0, 5), (0, 0, -1))
    assert hit and t == 4.5
    # just outside: the world box passes (vd == 0 skips the axis, bbox.cc:48-49)
    # but the local test misses
    hit, *_ = _probe(pkg, orc, "box.ray", (0.5000001, 0, 5), (0, 0, -1))
    assert not hit


def test_kat_cylinder(pkg, orc):
    hit, t, n, _, _ = _probe(pkg, orc, "cylinder.ray", (0, 0, 5), (0, 0, -1))
    assert hit and t == 4.0 and n == (0.0, 0.0, 1.0)  # cap at z = 1
    hit, t, n, _, _ = _probe(pkg, orc, "cylinder.ray", (5, 0, 0.5), (-1, 0, 0))
    assert hit and t == 4.0 and n == (1.0, 0.0, 0.0)  # body


def test_kat_cone(pkg, orc):
    # default cone: bottom 1, top 0 -> 0.0001, height 1, capped (Parser.cpp:472-518,
    # Cone.h:11-37): beta = -0.9999, gamma = 0.0001 / beta - 1
    # on the axis the quadric has a double root: discriminant 0 -> miss, the
    # caps are never tested (Cone.cpp:31)
    hit, *_ = _probe(pkg, orc, "cone.ray", (0, 0, 5), (0, 0, -1))
    assert not hit
    # body at z = 0.5: radius 0.9999 * 0.50010001 = 0.50005
    hit, t, n, obj, face = _probe(pkg, orc, "cone.ray", (5, 0, 0.5), (-1, 0, 0))
    assert hit and abs(t - 4.49995) < 1e-12 and obj == 0 and face == -1
    nn = np.array([0.50005, 0.0, 2 * 0.9999 ** 2 * 0.50010001])
    assert np.abs(np.array(n) - nn / np.linalg.norm(nn)).max() < 1e-12
    # from below, off axis: the bottom cap (t = 5) beats the body root (5.50005)
    hit, t, n, _, _ = _probe(pkg, orc, "cone.ray", (0.5, 0, -5), (0, 0, 1))
    assert hit and t == 5.0 and n == (0.0, 0.0, -1.0)


def test_kat_cone_uncapped_quirks(pkg, orc):
    # bottom 1, top 0.5, height 2: beta = -0.25, gamma = 0.5 / beta - 2 = -4
    hit, t, n, _, _ = _probe(pkg, orc, "cone_open.ray", (5, 0, 0.5), (-1, 0, 0))
    assert hit and t == 4.125
    nn = np.array([0.875, 0.0, 0.4375])
    assert np.abs(np.array(n) - nn / np.linalg.norm(nn)).max() < 1e-15
    # from inside: the far root (-0.875) replaces the near one because it is
    # good and below theRoot (Cone.cpp:48), then theRoot <= RAY_EPSILON: the
    # closest-hit query misses ...
    hit, *_ = _probe(pkg, orc, "cone_open.ray", (0, 0, 0.5), (1, 0, 0))
    assert not hit
    # ... while intersectLocalList keeps the near root (shadow walks see it)
    path = os.path.join(KAT, "cone_open.ray")
    t, o, f, nh = orc.query_batch(pkg, path, np.array([[0.0, 0.0, 0.5]]), np.array([[1.0, 0.0, 0.0]]), 1, 4)
    assert nh[0] == 1 and t[0, 0] == 0.875 and o[0, 0] == 0


def test_kat_triangle_edges(pkg, orc):
    hit, t, n, obj, face = _probe(pkg, orc, "triangle.ray", (0.25, 0.25, 1), (0, 0, -1))
    assert hit and t == 1.0 and n == (0.0, 0.0, 1.0) and face == 0
    # on an edge / a vertex: BTTC rejects < 3.125e-10 (trimesh.cpp:141, U11)
    for p in ((0.5, 0.0, 1.0), (0.0, 0.5, 1.0), (0.0, 0.0, 1.0)):
        hit, *_ = _probe(pkg, orc, "triangle.ray", p, (0, 0, -1))
        assert not hit, p
    # parallel ray: ZCHK
    hit, *_ = _probe(pkg, orc, "triangle.ray", (-1, 0.25, 0), (1, 0, 0))
    assert not hit


# ------------------------------------------------------------------ golden fixtures
def _golden_files():
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("oracle_") and f.endswith(".npz"))


@pytest.mark.parametrize("fname", _golden_files())
def test_oracle_matches_golden(pkg, orc, fname):
    g = np.load(os.path.join(GOLDEN, fname))
    opts = cli_opts(pkg, str(g["flags"]))
    r = orc.render(pkg, scene_path(str(g["scene"])), opts, want_hits=True)
    assert np.array_equal(r["rgb8"], g["rgb8"])
    np.testing.assert_allclose(r["rgb"], g["rgb"], rtol=0, atol=1e-12, equal_nan=True)  # -O o can give NaN
    for f in ("object", "face", "scene_leaf", "mesh_leaf", "nrays"):
        assert np.array_equal(r["hits"][f], g["hits"][f]), f
    assert r["stats"]["rays"] == int(g["rays"])


# ------------------------------------------------------------------ CLI
def test_cli_argument_errors():
    ray = os.path.join(PKG_DIR, "bin", "ray")
    r = subprocess.run([ray], capture_output=True, text=True)
    assert r.returncode == 1 and "no input" in r.stderr
    r = subprocess.run([ray, "-O", "z", "a.ray", "b.png"], capture_output=True, text=True)
    assert r.returncode == 1 and "Invalid argument for O" in r.stderr
    r = subprocess.run([ray, "-A", "3", "a.ray", "b.png"], capture_output=True, text=True)
    assert r.returncode == 1 and "Invalid argument for A" in r.stderr
    r = subprocess.run([ray, "/nonexistent.ray", "/tmp/x.png"], capture_output=True, text=True)
    assert r.returncode == 1 and "Unable to load ray file" in r.stderr


def test_cli_json_and_modes_parse(pkg, tmp_path):
    o = pkg.RenderOptions.from_cli("-w 64 -r 3 -O d -A 2.5 -B 16 -C 0.05 -O r -A 4 -O s -A 7 -O c -A 0.2".split())
    assert (o.width, o.depth, o.dof, o.dof_fd, o.dof_div, o.dof_apsz) == (64, 3, True, 2.5, 16, 0.05)
    assert (o.aa_mode, o.aa_samples, o.ss_res, o.aterm_thresh) == (pkg.RTX_AA_SUPERSAMPLE, 4, 7, 0.2)


def test_oracle_cli_writes_png(tmp_path):
    from PIL import Image

    exe = os.path.join(ROOT, "oracle", "_build", "ray_oracle")
    out = tmp_path / "o.png"
    r = subprocess.run([exe, "-w", "40", "-r", "2", os.path.join(NEWSCENE, "spheres_overlap.ray"), str(out)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    im = Image.open(out)
    assert im.size == (40, 40) and im.mode == "RGB"


def test_png_rows_flipped(pkg, tmp_path):
    """writePNG stores buffer row 0 as the bottom row (pngimage.cpp:264)."""
    from PIL import Image

    a = np.zeros((4, 3, 3), np.uint8)
    a[0, :, 0] = 255  # buffer row 0: red
    p = tmp_path / "f.png"
    pkg.write_image(str(p), a)
    im = np.asarray(Image.open(p))
    assert im[-1, 0, 0] == 255 and im[0, 0, 0] == 0
    pb = tmp_path / "f.bmp"
    pkg.write_image(str(pb), a)
    imb = np.asarray(Image.open(pb))
    assert imb[-1, 0, 0] == 255


# ------------------------------------------------------------------ PNG textures (f1)
FEATURE = os.path.join(GOLDEN, "feature")


def test_png_reader_matches_independent_fixtures(pkg):
    """readPNG (pngimage.cpp:195-216) with libpng's transforms: every colour
    type, bit depths 2/4/8/16, all five filters, Adam7, tRNS, gAMA — decoded
    pixels equal the values tools/gen_png_fixtures.py encoded (rows flipped,
    row 0 = bottom)."""
    exp = np.load(os.path.join(FEATURE, "png_expected.npz"))
    assert len(exp.files) >= 11
    for name in exp.files:
        got = pkg.read_image(os.path.join(FEATURE, name + ".png"))
        assert got.shape == exp[name].shape, name
        assert np.array_equal(got, exp[name]), name


def test_png_reader_rejects_bad_files(pkg, tmp_path):
    bad = tmp_path / "bad.png"
    bad.write_bytes(b"\x89PNG\r\n\x1a\nnot really")
    with pytest.raises(pkg.RtxError):
        pkg.read_image(str(bad))
    trunc = tmp_path / "trunc.png"
    trunc.write_bytes(open(os.path.join(FEATURE, "png_rgb8.png"), "rb").read()[:60])
    with pytest.raises(pkg.RtxError):
        pkg.read_image(str(trunc))
    with pytest.raises(pkg.RtxError):
        pkg.read_image(str(tmp_path / "missing.png"))


def test_png_texture_scene_loads(pkg):
    # vec3 map paths are relative to the scene file (Parser.cpp:1276-1308)
    h = pkg.HostScene(os.path.join(FEATURE, "png_tex.ray"))
    assert h.info.n_textures == 5


# ------------------------------------------------------------------ 1M-face dragon BVH (f3)
def test_dragon_bvh_matches_restated_kdtree(pkg, orc, tmp_path_factory):
    """Parser + KdTree build for the 1M-triangle C5 scene (Parser.cpp:520-671,
    kdTree.h:27-78): the product's flattened trees hash identically to the
    restatement's pointer KdTrees (951,423 mesh nodes, depth 19)."""
    d = tmp_path_factory.mktemp("dragon")
    subprocess.run(["python3", os.path.join(ROOT, "tools", "gen_scenes.py"), str(d), "--dragon"], check=True,
                   capture_output=True)
    path = os.path.join(str(d), "dragon.ray")
    h = pkg.HostScene(path)
    assert h.info.n_faces == 1000000
    assert h.info.n_mesh_nodes == 951423
    assert h.info.mesh_depth == 19
    sh, mh = orc.bvh_hash(pkg, path)
    assert (h.info.scene_bvh_hash, h.info.mesh_bvh_hash) == (sh, mh)


# ------------------------------------------------------------------ oracle independence
class _RtxObject(C.Structure):
    _fields_ = [("wmin", C.c_double * 3), ("wmax", C.c_double * 3), ("inv", C.c_double * 12),
                ("normi", C.c_double * 9), ("type", C.c_int32), ("material", C.c_int32), ("mesh", C.c_int32),
                ("orig_id", C.c_int32), ("leaf", C.c_int32), ("pad", C.c_int32 * 5)]


def test_oracle_links_no_product_scene_build():
    """The checker restates the scene build itself: oracle/
    compiles neither glm_compat.cpp nor scene_build.cpp, and liboracle.so
    defines none of their symbols."""
    mk = open(os.path.join(ROOT, "oracle", "Makefile")).read()
    src = [ln for ln in mk.splitlines() if ln.startswith("SRC")][0]
    assert "glm_compat" not in src and "scene_build.cpp" not in src
    out = subprocess.run(["nm", "-C", "--defined-only", os.path.join(ROOT, "oracle", "_build", "liboracle.so")],
                         check=True, capture_output=True, text=True).stdout
    for sym in ("rtxh::mat4_inverse", "rtxh::finalize_scene", "rtxh::Camera::setLook", "rtxh::make_transform"):
        assert sym not in out, sym


SCENE_BUILD_CASES = ["xforms.ray", "xforms_quat.ray", "vmats.ray", "circ_light.ray", "png_tex.ray", "hitchcock.ray",
                     "trimesh2.ray", "spheres_overlap.ray", "distance.ray", "lava_box.ray", "concrete_2.ray",
                     "box_cyl_opaque_shadow_spotlight.ray", "cones.ray"]


@pytest.mark.parametrize("scene", SCENE_BUILD_CASES)
def test_scene_build_matches_restatement(pkg, orc, scene):
    """Product scene build (scene_build.cpp over glm_compat.cpp) vs the
    oracle's own restatement: world boxes, inverse rows, normi and the camera
    basis agree bit for bit."""
    path = scene_path(scene)
    h = pkg.HostScene(path)
    objs, cam = orc.scene_dump(pkg, path)
    n = h.desc.n_objects
    assert n == objs.shape[0]
    arr = (_RtxObject * n).from_address(h.desc.objects)
    got = np.zeros((n, 27))
    for o in arr:
        got[o.orig_id] = list(o.wmin) + list(o.wmax) + list(o.inv) + list(o.normi)
    assert np.array_equal(got.view(np.uint64), objs.view(np.uint64)), np.argwhere(got != objs)[:5]
    c = h.desc.camera
    pc = np.array([list(c.eye), list(c.look), list(c.u), list(c.v)])
    assert np.array_equal(pc.view(np.uint64), cam.view(np.uint64))


def test_kat_composed_transforms(pkg, orc):
    """translate(1, 2, -3, rotate(z, pi/2, scale(2, 1, 1, sphere))): an
    ellipsoid centred at (1, 2, -3) with semi-axis 2 along world y.  A ray
    down -y from y = 12 meets its top at y = 4 (t = 8); one along -z meets
    the front at z = -2 (t = 12)."""
    hit, t, n, obj, _ = _probe(pkg, orc, "xform_nested.ray", (1, 12, -3), (0, -1, 0))
    assert hit and abs(t - 8.0) < 1e-12 and np.abs(np.array(n) - [0, 1, 0]).max() < 1e-12
    hit, t, n, _, _ = _probe(pkg, orc, "xform_nested.ray", (1, 2, 10), (0, 0, -1))
    assert hit and abs(t - 12.0) < 1e-12 and np.abs(np.array(n) - [0, 0, 1]).max() < 1e-12
    hit, *_ = _probe(pkg, orc, "xform_nested.ray", (2.5, 2, 10), (0, 0, -1))  # |x - 1| > 1: outside
    assert not hit
    objs, cam = orc.scene_dump(pkg, os.path.join(KAT, "xform_nested.ray"))
    assert np.abs(objs[0, :6] - [0, 0, -4, 2, 4, -2]).max() < 1e-12  # world box
    # fov 90 with camera.cpp's PI = 3.14159265359: v = (0, 2 tan(pi/4), 0)
    assert cam[1].tolist() == [0.0, 0.0, -1.0] and abs(cam[3][1] - 2.0) < 1e-11


def test_kat_transform_matrix(pkg, orc):
    """transform((1,0,0,.5), (0,2,0,0), (0,0,1,-1), (0,0,0,1), box): rows as
    written (glm::transpose of the column constructor, Parser.cpp:313-346) —
    the unit box stretched 2x in y and centred at (0.5, 0, -1)."""
    hit, t, n, _, _ = _probe(pkg, orc, "xform_matrix.ray", (0.5, 0, 5), (0, 0, -1))
    assert hit and t == 5.5 and n == (0.0, 0.0, 1.0)
    hit, t, n, _, _ = _probe(pkg, orc, "xform_matrix.ray", (0.5, 10, -1), (0, -1, 0))
    assert hit and t == 9.0 and n == (0.0, 1.0, 0.0)
    hit, *_ = _probe(pkg, orc, "xform_matrix.ray", (0.5, 1.01, 5), (0, 0, -1))
    assert not hit


def test_kat_per_vertex_materials(pkg, orc):
    """trimesh.cpp:157-163: a hit's material is Material() += b_k * M_k over
    the face's vertices — with ambient light 1 and nothing else, the colour
    at barycentric (u, v, w) is the interpolated ambient (ka = (u, v, w))."""
    opts = pkg.RenderOptions.from_cli("-w 16 -r 0".split())
    r = orc.render(pkg, os.path.join(KAT, "vmat_quad.ray"), opts, want_hits=True)
    # the camera looks at (0.25, 0.25) down -z: the pixel at the image centre
    # sees the triangle at (0.25 + dx, 0.25 + dy); ka = (1 - x - y, x, y)
    hit = r["hits"][..., 0]["object"] >= 0
    assert hit.sum() > 40
    rgb = r["rgb"][hit]
    assert np.abs(rgb.sum(axis=1) - 1.0).max() < 1e-12  # barycentric weights sum to 1
    assert (rgb >= -1e-12).all()


def test_oracle_O0_build_equals_O2(pkg, orc):
    """bench.py's -O0 context row times the restatement built at the
    reference's own optimisation level (ray/cmake/env.cmake:9): the same
    arithmetic (-ffp-contract=off, SSE2 doubles), so the same image and the
    same ray counts as the -O2 checker."""
    path = scene_path("hitchcock.ray")
    opts = cli_opts(pkg, "-w 48 -r 3 -O r -A 2")
    a = orc.render(pkg, path, opts, want_hits=False)
    b = orc.render(pkg, path, opts, want_hits=False, lib_path=orc.LIB_O0)
    assert np.array_equal(a["rgb"], b["rgb"])
    assert a["stats"]["rays"] == b["stats"]["rays"]
