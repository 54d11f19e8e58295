"""ctypes binding of oracle/_build/liboracle.so — the CPU restatement of the
reference path (see oracle.h).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / the timed CPU baseline.  The
product (librtx_hip.so, bin/ray) never uses it.  Parity vs the original
binary is UNPINNED (the reference cannot be built here: SURVEY.md 8(c)).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
LIB_O0 = os.path.join(HERE, "_build", "liboracle_O0.so")  # the reference's -O0 (bench context row)
CLI = os.path.join(HERE, "_build", "ray_oracle")

_libs = {}


def build(quiet: bool = True):
    subprocess.run(["make", "-C", HERE, "-j4"], check=True, capture_output=quiet)


class OracleRect(C.Structure):
    _fields_ = [("x0", C.c_int32), ("y0", C.c_int32), ("x1", C.c_int32), ("y1", C.c_int32),
                ("threads", C.c_int32)]


def lib(pkg, path: str = LIB):
    """Load liboracle.so (or its -O0 build, LIB_O0); `pkg` is the loaded
    cs378hgraphics-raytracer_amd module (for the shared struct definitions of
    rtx.h)."""
    if path not in _libs:
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_aspect.restype = C.c_double
        L.oracle_aspect.argtypes = [C.c_char_p]
        L.oracle_scene_dump.argtypes = [C.c_char_p, C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.c_void_p]
        L.oracle_render.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(pkg.RtxRenderParams), C.POINTER(OracleRect),
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(pkg.RtxStats)]
        L.oracle_bvh_hash.argtypes = [C.c_char_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.oracle_probe.argtypes = [C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                   C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                   C.POINTER(C.c_int32)]
        L.oracle_query_batch.argtypes = [C.c_char_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        for fn in (L.oracle_raw_records, L.oracle_tokens):
            fn.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
        _libs[path] = L
    return _libs[path]


def _text(fn, path: str) -> str:
    need = C.c_int64()
    if fn(path.encode(), None, 0, C.byref(need)) != 0:
        raise RuntimeError("oracle text query failed")
    buf = C.create_string_buffer(need.value)
    if fn(path.encode(), buf, need.value, C.byref(need)) != 0:
        raise RuntimeError("oracle text query failed")
    return buf.value.decode("latin-1")


def raw_records(pkg, path: str) -> str:
    """The raw parse records of the oracle's own loader (parse_restated.cpp),
    canonical text (csrc/host/raw_records.h); "ERROR\t<message>" on failure."""
    return _text(lib(pkg).oracle_raw_records, path)


def tokens(pkg, path: str) -> str:
    """The oracle tokenizer's stream (rtx_host_tokens format)."""
    return _text(lib(pkg).oracle_tokens, path)


def query_batch(pkg, path: str, P, D, mode: int, kmax: int = 1):
    """Scene::intersect (mode 0) or sorted intersectList (mode 1) for rays
    (P[k], D[k]).  Returns (t, object, face, nhits) arrays."""
    import numpy as np

    L = lib(pkg)
    P = np.ascontiguousarray(P, np.float64)
    D = np.ascontiguousarray(D, np.float64)
    n = P.shape[0]
    k = 1 if mode == 0 else kmax
    t = np.zeros((n, k), np.float64)
    o = np.zeros((n, k), np.int32)
    f = np.zeros((n, k), np.int32)
    nh = np.zeros(n, np.int32)
    rc = L.oracle_query_batch(path.encode(), n, P.ctypes.data, D.ctypes.data, mode, k, t.ctypes.data, o.ctypes.data,
                              f.ctypes.data, nh.ctypes.data)
    if rc != 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return t, o, f, nh


def height_for(pkg, path: str, width: int) -> int:
    """CommandLineUI.cpp:156: height = (int)(w / aspectRatio + 0.5), with the
    restated camera's aspect ratio."""
    a = lib(pkg).oracle_aspect(path.encode())
    if a < 0:
        raise RuntimeError(lib(pkg).oracle_last_error().decode())
    return int(width / a + 0.5)


def render(pkg, path: str, opts, rect=None, threads: int = 0, want_hits: bool = True, lib_path: str = LIB):
    """Render with the restatement.  Returns dict(rgb8, rgb, hits, stats) in
    the same layout as DeviceScene.render (full frame).  lib_path: LIB_O0 for
    the -O0 build."""
    L = lib(pkg, lib_path)
    h = height_for(pkg, path, opts.width)
    p = opts.params(h)
    w = opts.width
    rgb8 = np.zeros((h, w, 3), np.uint8)
    rgb = np.zeros((h, w, 3), np.float64)
    # np.zeros maps lazily: with a rect only the rect's rows are touched (a
    # band of the 3840x2160x64 C5 frame must not commit 17 GB of records)
    hits = np.zeros((h, w, opts.spp), pkg.HIT_DTYPE) if want_hits else None
    r = OracleRect(0, 0, 0, 0, threads)
    if rect is not None:
        r.x0, r.y0, r.x1, r.y1 = rect
    if hits is not None:
        if rect is not None:
            hits[rect[1]:rect[3], rect[0]:rect[2]]["object"] = -1
        else:
            hits["object"] = -1
    st = pkg.RtxStats()
    rc = L.oracle_render(path.encode(), opts.cubemap.encode(), C.byref(p), C.byref(r), rgb8.ctypes.data, rgb.ctypes.data,
                         hits.ctypes.data if hits is not None else None, C.byref(st))
    if rc != 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return {"rgb8": rgb8, "rgb": rgb, "hits": hits, "stats": st.as_dict(), "height": h, "width": w}


def scene_dump(pkg, path: str):
    """The restated scene build: (objects (n, 27) float64 — wmin, wmax,
    inverse rows 0..2 [c*3+r], normi [c*3+r] — and camera (4, 3): eye,
    look, u, v)."""
    L = lib(pkg)
    n = C.c_int32()
    cam = np.zeros((4, 3), np.float64)
    if L.oracle_scene_dump(path.encode(), None, 0, C.byref(n), cam.ctypes.data) != 0:
        raise RuntimeError(L.oracle_last_error().decode())
    objs = np.zeros((n.value, 27), np.float64)
    if L.oracle_scene_dump(path.encode(), objs.ctypes.data, n.value, C.byref(n), cam.ctypes.data) != 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return objs, cam


def bvh_hash(pkg, path: str):
    L = lib(pkg)
    a, b = C.c_uint64(), C.c_uint64()
    if L.oracle_bvh_hash(path.encode(), C.byref(a), C.byref(b)) != 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return a.value, b.value


def probe(pkg, path: str, p, d):
    L = lib(pkg)
    pp = (C.c_double * 3)(*p)
    dd = (C.c_double * 3)(*d)
    t = C.c_double()
    n = (C.c_double * 3)()
    o = C.c_int32()
    f = C.c_int32()
    rc = L.oracle_probe(path.encode(), pp, dd, C.byref(t), n, C.byref(o), C.byref(f))
    if rc < 0:
        raise RuntimeError(L.oracle_last_error().decode())
    return bool(rc), t.value, tuple(n), o.value, f.value
