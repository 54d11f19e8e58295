"""-c cube maps: the loader (TraceUI::smartLoadCubemap /
matchCubemapFiles, ui/TraceUI.cc:87-167) and the miss colour
(CubeMap::getColor, scene/cubeMap.cpp:12-44; RayTracer.cpp:167-169).

The reference ships no cube-map images; tests/golden/cubemap/ is made by
tools/gen_cubemap.py.  The miss colour is pinned by an independent numpy
restatement of getColor + TextureMap::getMappedValue (material.cpp:84-138)
over camera rays that hit nothing."""
import os
import shutil

import numpy as np

from conftest import GOLDEN, cli_opts

CUBE = os.path.join(GOLDEN, "cubemap")
FACES = ["posx", "negx", "posy", "negy", "posz", "negz"]
KAT = os.path.join(GOLDEN, "kat")


def _read_bmp(path):
    """24-bit BMP -> (h, w, 3) uint8 with row 0 = the file's first (bottom) row."""
    b = open(path, "rb").read()
    off = int.from_bytes(b[10:14], "little")
    w = int.from_bytes(b[18:22], "little", signed=True)
    h = int.from_bytes(b[22:26], "little", signed=True)
    stride = (w * 3 + 3) & ~3
    rows = np.frombuffer(b, np.uint8, count=stride * h, offset=off).reshape(h, stride)[:, :w * 3]
    return rows.reshape(h, w, 3)[..., ::-1].astype(np.float64)  # BGR -> RGB


def _mapped(tex, u, v):
    h, w, _ = tex.shape
    if not (0.0 <= u <= 1.0 and 0.0 <= v <= 1.0):
        return np.array([0.0, 1.0, 0.0])
    x, y = u * (w - 1), v * (h - 1)
    ix, iy = int(x), int(y)
    x -= ix
    y -= iy

    def px(a, b):
        return tex[b, a] if (0 <= a < w and 0 <= b < h) else np.zeros(3)

    rows = []
    for i in range(2):
        pl, pr = px(i + ix, iy), px(i + ix, 1 + iy)
        rows.append(y * (pr - pl) + pl)
    return (x * (rows[1] - rows[0]) + rows[0]) / 255.0


def _cube_color(faces, rd):
    a = np.abs(rd)
    xy, yz, zx = a[0] >= a[1], a[1] >= a[2], a[2] >= a[0]
    scale, d, m = 0.5, (0.0, 0.0), 0
    if xy and not zx:
        scale /= a[0]
        d, m = (rd[2] if rd[0] > 0 else -rd[2], rd[1]), (0 if rd[0] > 0 else 1)
    elif yz and not xy:
        scale /= a[1]
        d, m = (rd[0], rd[2] if rd[1] > 0 else -rd[2]), (2 if rd[1] > 0 else 3)
    elif zx and not yz:
        scale /= a[2]
        d, m = (rd[0] if rd[2] > 0 else -rd[0], rd[1]), (4 if rd[2] > 0 else 5)
    return _mapped(faces[m], d[0] * scale + 0.5, d[1] * scale + 0.5)


def test_loader_attaches_six_faces(pkg):
    h0 = pkg.HostScene(os.path.join(KAT, "sphere.ray"))
    h = pkg.HostScene(os.path.join(KAT, "sphere.ray"), cubemap=os.path.join(CUBE, "negy.bmp"))
    assert h.cubemap_error is None
    assert h.info.n_textures == h0.info.n_textures + 6
    assert list(h.desc.cubemap) == list(range(h0.info.n_textures, h0.info.n_textures + 6))
    assert list(h0.desc.cubemap) == [-1] * 6


def test_loader_errors_like_reference(pkg, tmp_path, capfd):
    sp = os.path.join(KAT, "sphere.ray")
    # no '/' in the name: pdir is the whole name, not a directory
    h = pkg.HostScene(sp, cubemap="posx.bmp")
    assert h.cubemap_error == "Couldn't open the directory posx.bmp"
    assert list(h.desc.cubemap) == [-1] * 6
    assert "Couldn't open the directory" in capfd.readouterr().err
    # five faces
    d = tmp_path / "five"
    d.mkdir()
    for f in FACES[:5]:
        shutil.copy(os.path.join(CUBE, f + ".bmp"), d / (f + ".bmp"))
    h = pkg.HostScene(sp, cubemap=str(d / "posx.bmp"))
    assert h.cubemap_error == "Cannot locate all six cubemap files"
    # two names that find_first_of gives the same face (any of 'p','o','s',
    # then an 'x'): a conflict whatever the directory order
    d = tmp_path / "clash"
    d.mkdir()
    shutil.copy(os.path.join(CUBE, "posx.bmp"), d / "px.bmp")
    shutil.copy(os.path.join(CUBE, "posx.bmp"), d / "sx.bmp")
    h = pkg.HostScene(sp, cubemap=str(d / "px.bmp"))
    assert h.cubemap_error is not None and "stop smartload to avoid confliction" in h.cubemap_error
    # an unreadable face
    d = tmp_path / "bad"
    d.mkdir()
    for f in FACES:
        (d / (f + ".bmp")).write_bytes(b"not a bitmap")
    h = pkg.HostScene(sp, cubemap=str(d / "posx.bmp"))
    assert h.cubemap_error is not None and h.cubemap_error.startswith("Unable to load texture map")


def test_miss_colour_matches_independent_restatement(pkg, orc):
    faces = [_read_bmp(os.path.join(CUBE, f + ".bmp")) for f in FACES]
    path = os.path.join(KAT, "sphere.ray")
    opts = cli_opts(pkg, "-w 16 -r 0 -c cubemap/posx.bmp")
    r = orc.render(pkg, path, opts, want_hits=True)
    host = pkg.HostScene(path)
    cam = host.desc.camera
    eye, look, u, v = (np.array(x[:]) for x in (cam.eye, cam.look, cam.u, cam.v))
    h, w = r["height"], r["width"]
    n_miss = 0
    for j in range(h):
        for i in range(w):
            if r["hits"][j, i, 0]["object"] >= 0:
                continue
            x, y = i / w - 0.5, j / h - 0.5
            d = look + x * u + y * v
            d = d * (1.0 / np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))
            want = np.clip(_cube_color(faces, d), 0.0, 1.0)
            assert np.abs(r["rgb"][j, i] - want).max() < 1e-12, (i, j)
            n_miss += 1
    assert n_miss > 100
    # without -c the misses are black
    r0 = orc.render(pkg, path, cli_opts(pkg, "-w 16 -r 0"), want_hits=True)
    miss = r0["hits"]["object"][..., 0] < 0
    assert np.all(r0["rgb"][miss] == 0.0)
