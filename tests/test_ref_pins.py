"""Pins from the reference itself: its tokenizer and image I/O, compiled
UNMODIFIED from /root/reference/ray/src (oracle/Makefile `ref`,
oracle/ref_harness.cpp -> oracle/_ref/libref_io.so), against the product's
own (librtx_host.so):

* the token stream and every scalar of each .ray fixture, and of edge-case
  texts, equal the product tokenizer's (Tokenizer.cpp:39-237, Token.cpp);
* readImage of every BMP / PNG fixture equals rtx_read_image byte for byte
  (bitmap.cpp:17-93, pngimage.cpp:195-216 with the image's own libpng 1.6);
* writeImage and rtx_write_image produce the same BMP bytes, and PNGs that
  both readers decode to the same pixels (pngimage.cpp:226-285).

Build container only: /root/reference does not exist on the GPU box, so
these tests skip there."""
import ctypes as C
import glob
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

REF_SRC = "/root/reference/ray/src"
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libref_io.so")

pytestmark = pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference sources absent (GPU box)")


@pytest.fixture(scope="module")
def ref():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True, capture_output=True)
    L = C.CDLL(REF_LIB)
    L.ref_tokens.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
    L.ref_read_image.argtypes = [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                 C.c_void_p, C.c_int64]
    L.ref_write_image.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.c_void_p]
    L.ref_last_error.restype = C.c_char_p
    return L


@pytest.fixture(scope="module")
def host(pkg):
    L = pkg.host_lib()
    L.rtx_host_tokens.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
    return L


def _tokens(fn, path):
    n = C.c_int64()
    assert fn(path.encode(), None, 0, C.byref(n)) == 0
    b = C.create_string_buffer(n.value)
    assert fn(path.encode(), b, n.value, C.byref(n)) == 0
    return b.value.decode(errors="replace").splitlines()


def _ray_fixtures():
    out = sorted(glob.glob(os.path.join(GOLDEN, "**", "*.ray"), recursive=True))
    out += sorted(p for p in glob.glob(os.path.join(ROOT, "scenes", "*.ray")) if not p.endswith("dragon.ray"))
    return out


@pytest.fixture(scope="module")
def orc_tokens(pkg, orc):
    orc.lib(pkg)
    return orc.lib(pkg).oracle_tokens


@pytest.mark.parametrize("path", _ray_fixtures(), ids=lambda p: os.path.relpath(p, ROOT))
def test_token_stream_matches_reference(ref, host, orc_tokens, path):
    """Both tokenizers, the product's (parser.cpp) and the checker's own
    (oracle/parse_restated.cpp), against the reference's."""
    want = _tokens(ref.ref_tokens, path)
    assert want[-1] == "EOF"
    assert _tokens(host.rtx_host_tokens, path) == want
    assert _tokens(orc_tokens, path) == want


# edge cases of the scanner: comments, quoted identifiers, aliases, scalars
# atof reads partially ('1-2', '1e', '--3', '.'), identifiers with '-',
# reserved words without names in getNameForToken, syntax errors
EDGE_TEXTS = {
    "comments": "SBT-raytracer 1.0\n// line comment\n/* block\n comment */ camera { fov = 30; }\n",
    "scalars": "1 -2 .5 -.25 1e3 1e-3 1e 1-2 --3 . 3.14159265358979323846 1e400 -0 007\n",
    "idents": 'foo _bar a-b-c "quoted name" "with space" colour polymesh gennormals fov x1y2\n',
    "punct": "( ) { } , = ;\n",
    "no_newline_at_eof": "sphere { material = { diffuse = (0.1, 0.2, 0.3); } }",
    "crlf": "SBT-raytracer 1.0\r\ncamera {\r\n position = (1,2,3);\r\n}\r\n",
    "unterminated_string": 'name = "oops\n',
    "unterminated_comment": "camera /* never closed\n",
    "bad_char": "camera { position = (1, 2, 3) } @\n",
    "slash_alone": "camera / 3\n",
    "empty": "",
}


@pytest.mark.parametrize("name", list(EDGE_TEXTS))
def test_token_edge_cases_match_reference(ref, host, orc_tokens, tmp_path, name):
    p = tmp_path / f"{name}.ray"
    p.write_bytes(EDGE_TEXTS[name].encode())
    want = _tokens(ref.ref_tokens, str(p))
    assert _tokens(host.rtx_host_tokens, str(p)) == want
    assert _tokens(orc_tokens, str(p)) == want


def _read(host, path):
    """rtx_read_image: (h, w, channels)"""
    w, h, ch = C.c_int32(), C.c_int32(), C.c_int32()
    if host.rtx_read_image(path.encode(), C.byref(w), C.byref(h), C.byref(ch), None, 0) != 0:
        return None
    out = np.zeros(w.value * h.value * ch.value, np.uint8)
    assert host.rtx_read_image(path.encode(), C.byref(w), C.byref(h), C.byref(ch), out.ctypes.data, out.size) == 0
    return out.reshape(h.value, w.value, ch.value)


def _ref_read(ref, path):
    """readImage: the pixels (h, w, channels).  readBMP's vector is height *
    padded-row bytes long with the pixels packed at the front (bitmap.cpp:
    57-91) — what TextureMap::getPixelAt reads, (x + y * width) * 3
    (material.cpp:128-132); readPNG's is exactly rowbytes * height."""
    w, h, n = C.c_int32(), C.c_int32(), C.c_int64()
    if ref.ref_read_image(path.encode(), C.byref(w), C.byref(h), C.byref(n), None, 0) != 0:
        return None
    out = np.zeros(n.value, np.uint8)
    assert ref.ref_read_image(path.encode(), C.byref(w), C.byref(h), C.byref(n), out.ctypes.data, out.size) == 0
    npx = w.value * h.value
    ch = 3 if path.lower().endswith(".bmp") else n.value // npx
    return out[: npx * ch].reshape(h.value, w.value, ch)


def _image_fixtures():
    return sorted(glob.glob(os.path.join(GOLDEN, "**", "*.bmp"), recursive=True) +
                  glob.glob(os.path.join(GOLDEN, "**", "*.png"), recursive=True))


@pytest.mark.parametrize("path", _image_fixtures(), ids=lambda p: os.path.relpath(p, GOLDEN))
def test_read_image_matches_reference(ref, host, path):
    want = _ref_read(ref, path)
    got = _read(host, path)
    assert want is not None, ref.ref_last_error()
    assert got is not None
    assert got.shape == want.shape
    assert np.array_equal(got, want), f"{int((got != want).sum())} bytes differ"


@pytest.mark.parametrize("ext", [".bmp", ".png"])
@pytest.mark.parametrize("w,h", [(1, 1), (3, 2), (37, 19), (64, 64)])
def test_write_image_matches_reference(ref, host, tmp_path, ext, w, h):
    rgb = np.random.default_rng(w * 1000 + h).integers(0, 256, (h, w, 3), dtype=np.uint8)
    a, b = str(tmp_path / f"ref{ext}"), str(tmp_path / f"rtx{ext}")
    assert ref.ref_write_image(a.encode(), w, h, rgb.ctypes.data) == 0
    assert host.rtx_write_image(b.encode(), w, h, rgb.ctypes.data) == 0
    if ext == ".bmp":
        fa, fb = open(a, "rb").read(), open(b, "rb").read()
        assert len(fa) == len(fb)
        # byte for byte, except the last row's padding: writeBMP copies the
        # padded row length from the packed buffer (bitmap.cpp:137), i.e.
        # reads past its end there (undefined; decision U25: zeros)
        pad = (4 - w * 3 % 4) % 4
        n = len(fa) - pad
        assert fa[:n] == fb[:n]
        assert fb[n:] == bytes(pad)
    for path in (a, b):
        ri, hi = _ref_read(ref, path), _read(host, path)
        assert ri is not None and hi is not None and np.array_equal(hi, ri)
        if ext == ".png":  # the buffer the writer was given
            assert np.array_equal(hi, rgb)
        # (readBMP compacts padded rows in place with out = in - offset, and
        # where the offset is 1 byte `out[1] = in[1]` overwrites in[0] before
        # `out[2] = in[0]` reads it (bitmap.cpp:76-90): such rows read back
        # with a wrong third channel — in the reference and here alike)
