"""The checker's own .ray loader (oracle/parse_restated.cpp, a restatement of
ray/src/parser/{Parser,Tokenizer,Token}.cpp and fileio/buffer.cpp) against the
product's (csrc/host/parser.cpp): VERDICT r03 item 5.  The oracle no longer
links the product parser, so a parse-semantics error above the token stream
(transform-chain order, material inheritance, scale(s) vs scale(x, y, z),
camera attribute order, light defaults) would now show up here as a raw
record mismatch instead of being shared by checker and product.

Both loaders print their raw records through the same canonical printer
(csrc/host/raw_records.h: a printer only, no parse semantics): every .ray
fixture must give identical text, and every malformed input the same
"ERROR\\t<RayTracer::loadScene message>" line."""
import ctypes as C
import glob
import os
import subprocess

import pytest

from conftest import FEATURE, GOLDEN, NEWSCENE, ROOT, SCENES

KAT = os.path.join(GOLDEN, "kat")


def _host_text(pkg, fn, path):
    L = pkg.host_lib()
    f = getattr(L, fn)
    f.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
    need = C.c_int64()
    assert f(path.encode(), None, 0, C.byref(need)) == 0
    buf = C.create_string_buffer(need.value)
    assert f(path.encode(), buf, need.value, C.byref(need)) == 0
    return buf.value.decode("latin-1")


def _fixtures():
    out = []
    for d in (NEWSCENE, FEATURE, KAT, SCENES, os.path.join(GOLDEN, "textures")):
        out += sorted(glob.glob(os.path.join(d, "*.ray")))
    return [p for p in out if os.path.basename(p) != "dragon.ray"]  # (1M faces: the BVH hash test covers it)


@pytest.mark.parametrize("path", _fixtures(), ids=lambda p: os.path.relpath(p, ROOT))
def test_raw_records_match(pkg, orc, path):
    want = _host_text(pkg, "rtx_host_raw_records", path)
    got = orc.raw_records(pkg, path)
    assert not want.startswith("ERROR"), want
    assert got == want


@pytest.mark.parametrize("path", _fixtures(), ids=lambda p: os.path.relpath(p, ROOT))
def test_token_streams_match(pkg, orc, path):
    assert orc.tokens(pkg, path) == _host_text(pkg, "rtx_host_tokens", path)


# malformed inputs: the loaders must fail with the same message (and line)
BAD = {
    "version": "SBT-raytracer 1.2\n",
    "no_header": "sphere {}\n",
    "updir_missing": "SBT-raytracer 1.0\ncamera { viewdir = (0,0,-1); }\n",
    "viewdir_missing": "SBT-raytracer 1.0\ncamera {\n updir = (0,1,0);\n}\n",
    "camera_attr": "SBT-raytracer 1.0\ncamera { color = (1,1,1); }\n",
    "group_material": "SBT-raytracer 1.0\n{ material = { diffuse = (1,0,0); } sphere {} }\n",
    "named_ident": "SBT-raytracer 1.0\nmaterial = { name = m; diffuse = (1,0,0); }\nsphere { material = m; }\n",
    "redefined": "SBT-raytracer 1.0\nmaterial = { name = m; }\nmaterial = { name = m; }\n",
    "bad_face": "SBT-raytracer 1.0\ntrimesh { points = ((0,0,0),(1,0,0),(0,1,0)); faces = ((0,1,5)); }\n",
    "short_face": "SBT-raytracer 1.0\ntrimesh { points = ((0,0,0),(1,0,0),(0,1,0)); faces = ((0,1)); }\n",
    "wrong_normals": "SBT-raytracer 1.0\ntrimesh { points = ((0,0,0),(1,0,0),(0,1,0)); normals = ((0,0,1)); "
                     "faces = ((0,1,2)); }\n",
    "wrong_materials": "SBT-raytracer 1.0\ntrimesh { points = ((0,0,0),(1,0,0),(0,1,0)); "
                       "materials = ({ diffuse = (1,0,0); }); faces = ((0,1,2)); }\n",
    "texture": "SBT-raytracer 1.0\nsphere { material = { diffuse = map(\"nope.bmp\"); } }\n",
    "unknown_geometry": "SBT-raytracer 1.0\nteapot {}\n",
    "unterminated_comment": "SBT-raytracer 1.0\nsphere {} /* unterminated\n",
    "unexpected_char": "SBT-raytracer 1.0\nsphere {} ?\n",
    "unterminated_string": "SBT-raytracer 1.0\nsphere { name = \"abc\n}\n",
    "point_no_pos": "SBT-raytracer 1.0\npoint_light { color = (1,1,1); }\n",
    "point_repeat": "SBT-raytracer 1.0\npoint_light { color = (1,1,1); color = (1,1,1); }\n",
    "point_radius": "SBT-raytracer 1.0\npoint_light { radius = 1; }\n",
    "dir_no_dir": "SBT-raytracer 1.0\ndirectional_light { color = (1,1,1); }\n",
    "dir_atten": "SBT-raytracer 1.0\ndirectional_light { constant_attenuation_coeff = 1; }\n",
    "rect_no_updir": "SBT-raytracer 1.0\narea_light_rect { position = (0,0,0); direction = (0,0,1); "
                     "color = (1,1,1); width = 1; height = 1; }\n",
    "circ_no_radius": "SBT-raytracer 1.0\narea_light_circ { position = (0,0,0); direction = (0,0,1); "
                      "color = (1,1,1); }\n",
    "spot_no_angle": "SBT-raytracer 1.0\nspot_light { position = (0,0,0); direction = (0,0,1); radius = 1; "
                     "color = (1,1,1); }\n",
    "spot_width": "SBT-raytracer 1.0\nspot_light { width = 1; }\n",
    "cone_bool": "SBT-raytracer 1.0\ncone { capped = 1; }\n",
    "sphere_capped": "SBT-raytracer 1.0\nsphere { capped = true; }\n",
    "ambient_no_color": "SBT-raytracer 1.0\nambient_light { position = (1,1,1); }\n",
    "scale_two": "SBT-raytracer 1.0\nscale(2, 3, sphere {})\n",
    "translate_short": "SBT-raytracer 1.0\ntranslate(1, 2, sphere {})\n",
    "transform_rows": "SBT-raytracer 1.0\ntransform((1,0,0,0),(0,1,0,0),(0,0,1,0), sphere {})\n",
    "eof_in_group": "SBT-raytracer 1.0\n{ sphere {}\n",
    "eof_no_newline": "SBT-raytracer 1.0\nsphere {",
    "material_attr": "SBT-raytracer 1.0\nsphere { material = { colour = (1,1,1); } }\n",
    "trimesh_attr": "SBT-raytracer 1.0\ntrimesh { fov = 3; }\n",
    "gennormals_nosemi": "SBT-raytracer 1.0\ntrimesh { gennormals }\n",
    "bad_after_error": "SBT-raytracer 1.0\nsphere { } }\n ? ? ?\n",
    "empty": "",
}


@pytest.mark.parametrize("name", sorted(BAD))
def test_errors_match(pkg, orc, tmp_path, name):
    p = tmp_path / "bad.ray"
    p.write_text(BAD[name])
    want = _host_text(pkg, "rtx_host_raw_records", str(p))
    got = orc.raw_records(pkg, str(p))
    assert want.startswith("ERROR"), want
    assert got == want


# well-formed edge cases: quirks both loaders must reproduce the same way
GOOD = {
    "scale_uniform": "SBT-raytracer 1.0\nscale(2, sphere {});\nscale(1, 2, 3, box {})\n",
    "nested_chain": "SBT-raytracer 1.0\ntranslate(1,2,3, rotate(0,1,0,0.5, scale(2, { box {} "
                    "transform((1,0,0,1),(0,1,0,2),(0,0,1,3),(0,0,0,1), sphere {}) })))\n",
    "material_inherit": "SBT-raytracer 1.0\nmaterial = { diffuse = (1,0,0); reflective = (0.5,0.5,0.5); }\n"
                        "sphere {}\nmaterial = { specular = (1,1,1); }\nsphere { material = { index = 1.5; } }\n"
                        "box { material = { transmissive = map(\"tex.png\"); shininess = map(\"TEXDIR/tex.png\"); } }\n",
    "named_material": "SBT-raytracer 1.0\nmaterial = { name shiny; specular = (1,1,1); shininess = 64; }\n"
                      "sphere {}\n",
    "camera_order": "SBT-raytracer 1.0\ncamera { fov = 40; position = (1,2,3); quaternian = (1,0,0,0); "
                    "aspectratio = 2; viewdir = (0,0,-1); updir = (0,1,0); fov = 50; }\n"
                    "camera { aspectratio = 1.5 }\n",
    "lights_defaults": "SBT-raytracer 1.0\npoint_light { position = (0,1,0); colour = (1,1,1); }\n"
                       "point_light { position = (0,1,0); color = (1,1,1); quadratic_attenuation_coeff = 0.3; "
                       "constant_attenuation_coeff = 0.1 }\n"
                       "directional_light { direction = (0,-1,0); color = (0.5,0.5,0.5); }\n"
                       "ambient_light { color = (0.1,0.1,0.1); } ambient_light { color = (0.2,0.2,0.2); }\n",
    "cone_shapes": "SBT-raytracer 1.0\ncone { height = -2; bottom_radius = -0.5; top_radius = 0; capped = false; }\n"
                   "cone { top_radius = 1; }\ncone { height = 3; bottom_radius = 1.0005; top_radius = 1; }\n",
    "polymesh_fan": "SBT-raytracer 1.0\npolymesh { points = ((0,0,0),(1,0,0),(1,1,0),(0,1,0),(0.5,2,0)); "
                    "faces = ((0,1,2,3,4), (0.9,1.2,2.7)); gennormals; material = { diffuse = (0,1,0); }; "
                    "materials = ({ ambient = (1,0,0); }, { }, { }, { }, { diffuse = (0,0,1); }); }\n",
    "comments": "SBT-raytracer 1.0 // header\n/* block\n * comment */ sphere { name = \"a b\"; }\n"
                "// last line without newline",
    "scalars": "SBT-raytracer 1.0\ntranslate(1e2, -.5, 3.-2, sphere {})\n",
}


@pytest.mark.parametrize("name", sorted(GOOD))
def test_edge_cases_match(pkg, orc, tmp_path, name):
    d = tmp_path / "a" / "b"
    d.mkdir(parents=True)
    p = d / "edge.ray"
    import shutil

    shutil.copy(os.path.join(FEATURE, "png_tex_diffuse.png"), d / "tex.png")
    # a scalar parameter's map() path is taken as written (no base path)
    p.write_text(GOOD[name].replace("TEXDIR", str(d)))
    want = _host_text(pkg, "rtx_host_raw_records", str(p))
    got = orc.raw_records(pkg, str(p))
    assert not want.startswith("ERROR"), want
    assert got == want


def test_oracle_links_no_product_parser():
    """oracle/Makefile compiles parse_restated.cpp, not the product's
    parser.cpp, and liboracle.so defines none of its entry points."""
    mk = open(os.path.join(ROOT, "oracle", "Makefile")).read()
    src = [ln for ln in mk.splitlines() if ln.startswith("SRC")][0]
    assert "parser.cpp" not in src and "parse_restated.cpp" in src
    out = subprocess.run(["nm", "-C", "--defined-only", os.path.join(ROOT, "oracle", "_build", "liboracle.so")],
                         check=True, capture_output=True, text=True).stdout
    for sym in ("rtxh::parse_ray_file_raw", "rtxh::parse_ray_text", "rtxh::dump_ray_tokens", "rtxh::load_cubemap"):
        assert sym not in out, sym
