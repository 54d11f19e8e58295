"""cs378hgraphics-raytracer_amd — MI355X (gfx950) hot path of the reference
ray tracer (AlterionX/cs378hgraphics-raytracer), reached through its C ABI.

This module is a thin ctypes binding of include/rtx.h (librtx_hip.so) and
include/rtx_host.h (librtx_host.so).  It mirrors the reference's RayTracer
interface (ray/src/RayTracer.h:26-75): ``Scene.load`` == RayTracer::loadScene,
``Scene.render`` == traceSetup + traceImage + getBuffer.  There is no CPU
fallback: importing works anywhere, but rendering needs a gfx950 device and
raises ``RtxError`` otherwise.

The package directory name contains '-', so load it with
``load_package()`` from the repo root helpers or importlib.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
BIN_DIR = os.path.join(PKG_DIR, "bin")
REPO_ROOT = os.path.dirname(PKG_DIR)

RTX_AA_NONE, RTX_AA_SUPERSAMPLE, RTX_AA_ADAPTIVE, RTX_AA_JITTERED = 0, 1, 2, 3
RTX_OK, RTX_ERR_INVALID, RTX_ERR_HIP, RTX_ERR_NODEVICE, RTX_ERR_CAPACITY, RTX_ERR_FRAME = 0, -1, -2, -3, -4, -5  # include/rtx.h


class RtxError(RuntimeError):
    pass


# ---------------------------------------------------------------- structs (rtx.h)
class RtxCamera(C.Structure):
    _fields_ = [("eye", C.c_double * 3), ("look", C.c_double * 3), ("u", C.c_double * 3),
                ("v", C.c_double * 3), ("aspect", C.c_double)]


class RtxSceneDesc(C.Structure):
    _fields_ = [
        ("scene_nodes", C.c_void_p), ("n_scene_nodes", C.c_int32),
        ("objects", C.c_void_p), ("n_objects", C.c_int32),
        ("materials", C.c_void_p), ("n_materials", C.c_int32),
        ("meshes", C.c_void_p), ("n_meshes", C.c_int32),
        ("mesh_nodes", C.c_void_p), ("n_mesh_nodes", C.c_int32),
        ("faces", C.c_void_p), ("n_faces", C.c_int32),
        ("face_ids", C.c_void_p),
        ("vnormals", C.c_void_p), ("n_vnormals", C.c_int32),
        ("vmats", C.c_void_p), ("n_vmats", C.c_int32),
        ("lights", C.c_void_p), ("n_lights", C.c_int32),
        ("textures", C.c_void_p), ("n_textures", C.c_int32),
        ("texels", C.c_void_p), ("n_texels", C.c_int64),
        ("camera", RtxCamera),
        ("ambient", C.c_double * 3),
        ("scene_depth", C.c_int32),
        ("mesh_depth", C.c_int32),
        ("obj_params", C.c_void_p),
        ("cubemap", C.c_int32 * 6),
    ]


class RtxRenderParams(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("depth", C.c_int32), ("aa_mode", C.c_int32),
        ("aa_samples", C.c_int32), ("dof", C.c_int32), ("dof_div", C.c_int32), ("anaglyph", C.c_int32),
        ("ss_res", C.c_int32), ("overlapping", C.c_int32),
        ("aa_thresh", C.c_double), ("aterm_thresh", C.c_double), ("dof_fd", C.c_double), ("dof_apsz", C.c_double),
        ("tile", C.c_int32), ("shard", C.c_int32), ("nshards", C.c_int32), ("packed", C.c_int32),
    ]


class RtxHitRecord(C.Structure):
    _fields_ = [("object", C.c_int32), ("face", C.c_int32), ("scene_leaf", C.c_int32), ("mesh_leaf", C.c_int32),
                ("nrays", C.c_int32), ("pad", C.c_int32), ("t", C.c_double)]


HIT_DTYPE = np.dtype([("object", "<i4"), ("face", "<i4"), ("scene_leaf", "<i4"), ("mesh_leaf", "<i4"),
                      ("nrays", "<i4"), ("pad", "<i4"), ("t", "<f8")])
assert HIT_DTYPE.itemsize == C.sizeof(RtxHitRecord)


class RtxStats(C.Structure):
    _fields_ = [("rays", C.c_int64), ("camera_rays", C.c_int64), ("secondary_rays", C.c_int64),
                ("shadow_rays", C.c_int64), ("node_visits", C.c_int64), ("object_tests", C.c_int64),
                ("tri_tests", C.c_int64), ("shades", C.c_int64), ("kernel_ms", C.c_double),
                ("shadow_traced", C.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class RtxHostInfo(C.Structure):
    _fields_ = [("n_objects", C.c_int32), ("n_lights", C.c_int32), ("n_meshes", C.c_int32),
                ("n_faces", C.c_int32), ("n_textures", C.c_int32), ("n_scene_nodes", C.c_int32),
                ("n_mesh_nodes", C.c_int32), ("scene_depth", C.c_int32), ("mesh_depth", C.c_int32),
                ("n_cones", C.c_int32), ("n_area_lights", C.c_int32), ("aspect", C.c_double),
                ("scene_bvh_hash", C.c_uint64), ("mesh_bvh_hash", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# ---------------------------------------------------------------- library loading
_host = None
_hip = None


def host_lib():
    """librtx_host.so (parser, BVH build, flattening, image writer)."""
    global _host
    if _host is None:
        path = os.path.join(LIB_DIR, "librtx_host.so")
        if not os.path.exists(path):
            raise RtxError(f"{path} not built (run __graft_entry__.build())")
        lib = C.CDLL(path)
        lib.rtx_host_last_error.restype = C.c_char_p
        lib.rtx_host_load.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        lib.rtx_host_desc.argtypes = [C.c_void_p, C.POINTER(RtxSceneDesc)]
        lib.rtx_host_info.argtypes = [C.c_void_p, C.POINTER(RtxHostInfo)]
        lib.rtx_host_free.argtypes = [C.c_void_p]
        lib.rtx_host_cubemap.argtypes = [C.c_void_p, C.c_char_p]
        lib.rtx_write_image.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.c_void_p]
        lib.rtx_image_height.argtypes = [C.c_int32, C.c_double]
        lib.rtx_image_height.restype = C.c_int32
        lib.rtx_read_image.argtypes = [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                       C.POINTER(C.c_int32), C.c_void_p, C.c_int64]
        lib.rtx_shard_tiles.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                        C.c_int32, C.POINTER(C.c_int32)]
        lib.rtx_host_tokens.argtypes = [C.c_char_p, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
        lib.rtx_unpack_tiles.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                         C.c_int32, C.c_void_p]
        _host = lib
    return _host


def hip_lib():
    """librtx_hip.so (gfx950 kernels).  Raises if it is not built."""
    global _hip
    if _hip is None:
        # RTX_HIP_LIB: an alternative in-tree build of the same library
        # (tuning experiments, tools/build_variants.sh)
        path = os.environ.get("RTX_HIP_LIB") or os.path.join(LIB_DIR, "librtx_hip.so")
        if not os.path.exists(path):
            raise RtxError(f"{path} not built (run __graft_entry__.build()); there is no CPU fallback")
        lib = C.CDLL(path)
        lib.rtx_last_error.restype = C.c_char_p
        lib.rtx_device_count.argtypes = [C.POINTER(C.c_int)]
        lib.rtx_scene_create.argtypes = [C.c_int, C.POINTER(RtxSceneDesc), C.POINTER(C.c_void_p)]
        lib.rtx_scene_destroy.argtypes = [C.c_void_p]
        lib.rtx_render.argtypes = [C.c_void_p, C.POINTER(RtxRenderParams), C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_int, C.c_void_p, C.POINTER(RtxStats)]
        lib.rtx_shard_pixels.argtypes = [C.POINTER(RtxRenderParams), C.POINTER(C.c_int64)]
        lib.rtx_kernel_time.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int)]
        lib.rtx_last_work.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.c_int]
        lib.rtx_frame_status.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        lib.rtx_overlap_count.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        lib.rtx_frame_contexts.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
        _hip = lib
    return _hip


# symbols include/*.h declare (checked by the CPU test suite)
HIP_SYMBOLS = ["rtx_last_error", "rtx_device_count", "rtx_scene_create", "rtx_scene_destroy", "rtx_render",
               "rtx_shard_pixels", "rtx_kernel_time", "rtx_last_work", "rtx_frame_status", "rtx_overlap_count",
               "rtx_frame_contexts"]
HOST_SYMBOLS = ["rtx_host_last_error", "rtx_host_load", "rtx_host_desc", "rtx_host_info", "rtx_host_free",
                "rtx_host_cubemap", "rtx_write_image", "rtx_image_height", "rtx_read_image", "rtx_shard_tiles",
                "rtx_unpack_tiles", "rtx_host_tokens", "rtx_host_raw_records"]


def _check_host(rc, what):
    if rc != 0:
        raise RtxError(f"{what}: {host_lib().rtx_host_last_error().decode(errors='replace')} (status {rc})")


def _check(rc, lib, what):
    if rc != 0:
        raise RtxError(f"{what}: {lib.rtx_last_error().decode(errors='replace')} (status {rc})")


# ---------------------------------------------------------------- render options
@dataclass
class RenderOptions:
    """TraceUI flags (ui/TraceUI.h:34-129) with the reference defaults."""
    width: int = 512
    depth: int = 0
    aa_mode: int = RTX_AA_NONE
    aa_samples: int = 3
    aa_thresh: float = 1.0
    aterm_thresh: float = 0.0
    dof: bool = False
    dof_fd: float = 3.0
    dof_div: int = 5
    dof_apsz: float = 0.05
    anaglyph: bool = False
    ss_res: int = 5
    overlapping: bool = False
    cubemap: str = ""  # -c: one of the six cube-face files (CommandLineUI.cpp:41-42)

    @classmethod
    def from_cli(cls, args):
        """Parse reference CLI flags (-r -w -O -A -B -C; CommandLineUI.cpp:30-132)."""
        o = cls()
        prev = None
        it = iter(args)
        for a in it:
            if a == "-r":
                o.depth = int(next(it))
            elif a == "-w":
                o.width = int(next(it))
            elif a == "-c":
                o.cubemap = next(it)
            elif a == "-O":
                prev = next(it)[0]
                if prev == "a":
                    o.aa_mode = RTX_AA_ADAPTIVE
                elif prev == "j":
                    o.aa_mode = RTX_AA_JITTERED
                elif prev == "r":
                    o.aa_mode = RTX_AA_SUPERSAMPLE
                elif prev == "o":
                    o.overlapping = True
                elif prev == "d":
                    o.dof = True
                elif prev == "g":
                    o.anaglyph = True
                elif prev not in ("c", "s"):
                    raise ValueError(f"invalid -O {prev}")
            elif a == "-A":
                v = next(it)
                if prev in ("a", "j", "r"):
                    o.aa_samples = int(v)
                elif prev == "c":
                    o.aterm_thresh = float(v)
                elif prev == "d":
                    o.dof_fd = float(v)
                elif prev == "s":
                    o.ss_res = int(v)
                else:
                    raise ValueError("invalid -A")
            elif a == "-B":
                v = next(it)
                if prev == "a":
                    o.aa_thresh = float(v)
                elif prev == "d":
                    o.dof_div = int(v)
                else:
                    raise ValueError("invalid -B")
            elif a == "-C":
                v = next(it)
                if prev == "d":
                    o.dof_apsz = float(v)
                else:
                    raise ValueError("invalid -C")
            else:
                raise ValueError(f"unknown flag {a}")
        return o

    @property
    def spp(self) -> int:
        return 1 if self.aa_mode == RTX_AA_NONE else self.aa_samples * self.aa_samples

    def params(self, height: int, tile: int = 0, shard: int = 0, nshards: int = 1, packed: bool = False):
        p = RtxRenderParams()
        p.width, p.height, p.depth = self.width, height, self.depth
        p.aa_mode, p.aa_samples, p.aa_thresh = self.aa_mode, self.aa_samples, self.aa_thresh
        p.aterm_thresh = self.aterm_thresh
        p.dof, p.dof_fd, p.dof_div, p.dof_apsz = int(self.dof), self.dof_fd, self.dof_div, self.dof_apsz
        p.anaglyph, p.ss_res, p.overlapping = int(self.anaglyph), self.ss_res, int(self.overlapping)
        p.tile, p.shard, p.nshards, p.packed = tile, shard, nshards, int(packed)
        return p


# ---------------------------------------------------------------- scene
class HostScene:
    """A parsed + flattened scene (RayTracer::loadScene)."""

    def __init__(self, path: str, cubemap: str = ""):
        lib = host_lib()
        h = C.c_void_p()
        rc = lib.rtx_host_load(path.encode(), C.byref(h))
        if rc != 0:
            raise RtxError(lib.rtx_host_last_error().decode(errors="replace"))
        self._h = h
        self.path = path
        self.cubemap_error = None
        if cubemap:
            # TraceUI::smartLoadCubemap: a failure is reported on stderr and
            # the render goes on without a cube map
            if lib.rtx_host_cubemap(h, cubemap.encode()) != 0:
                self.cubemap_error = lib.rtx_host_last_error().decode(errors="replace")
                sys.stderr.write(self.cubemap_error + "\n")
        self.info = RtxHostInfo()
        lib.rtx_host_info(h, C.byref(self.info))
        self.desc = RtxSceneDesc()
        lib.rtx_host_desc(h, C.byref(self.desc))

    @property
    def aspect(self) -> float:
        return self.info.aspect

    def height_for(self, width: int) -> int:
        return int(host_lib().rtx_image_height(width, self.aspect))

    def close(self):
        if self._h:
            host_lib().rtx_host_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceScene:
    """Scene resident in HBM (rtx_scene_create)."""

    def __init__(self, host: HostScene, device: int = 0):
        lib = hip_lib()
        s = C.c_void_p()
        _check(lib.rtx_scene_create(device, C.byref(host.desc), C.byref(s)), lib, "rtx_scene_create")
        self._s = s
        self.host = host
        self.device = device

    def render(self, opts: RenderOptions, want_f64: bool = True, want_hits: bool = False, stats: bool = False,
               tile: int = 0, shard: int = 0, nshards: int = 1, packed: bool = False):
        """Synchronous render into host numpy arrays.  Returns dict with
        rgb8 (h, w, 3) uint8 in reference buffer order (row 0 = bottom),
        rgb (h, w, 3) float64, hits (h, w, spp) records, stats dict."""
        lib = hip_lib()
        h = self.host.height_for(opts.width)
        p = opts.params(h, tile, shard, nshards, packed)
        npix = C.c_int64()
        lib.rtx_shard_pixels(C.byref(p), C.byref(npix))
        n = npix.value
        rgb8 = np.zeros(n * 3, np.uint8)
        rgbf = np.zeros(n * 3, np.float64) if want_f64 else None
        hits = np.zeros(n * opts.spp, HIT_DTYPE) if want_hits else None
        st = RtxStats()
        rc = lib.rtx_render(self._s, C.byref(p), rgb8.ctypes.data,
                            rgbf.ctypes.data if rgbf is not None else None,
                            hits.ctypes.data if hits is not None else None, 0, None,
                            C.byref(st) if stats else None)
        _check(rc, lib, "rtx_render")
        out = {"height": h, "width": opts.width, "npix": n}
        if packed and tile:
            out["rgb8"], out["rgb"], out["hits"] = rgb8, rgbf, hits
        else:
            out["rgb8"] = rgb8.reshape(h, opts.width, 3)
            out["rgb"] = rgbf.reshape(h, opts.width, 3) if rgbf is not None else None
            out["hits"] = hits.reshape(h, opts.width, opts.spp) if hits is not None else None
        out["stats"] = st.as_dict() if stats else None
        if stats:
            out["stats"]["kernels"] = self.last_work()
        return out

    def render_device(self, opts: RenderOptions, rgb8_ptr: int, rgbf_ptr: int = 0, stream: int = 0,
                      tile: int = 0, shard: int = 0, nshards: int = 1, packed: bool = False):
        """Asynchronous render into device buffers (e.g. torch tensor
        data_ptr()) on the given hipStream_t."""
        lib = hip_lib()
        h = self.host.height_for(opts.width)
        p = opts.params(h, tile, shard, nshards, packed)
        rc = lib.rtx_render(self._s, C.byref(p), C.c_void_p(rgb8_ptr) if rgb8_ptr else None,
                            C.c_void_p(rgbf_ptr) if rgbf_ptr else None, None, 1,
                            C.c_void_p(stream) if stream else None, None)
        _check(rc, lib, "rtx_render")

    # rtx_last_work's kernel classes (include/rtx.h)
    WORK_CLASSES = ("closest", "next", "tail")
    WORK_FIELDS = ("queries", "node_visits", "object_tests", "tri_tests", "shades")

    def last_work(self):
        """Per-kernel-class work of the last render with stats=True:
        {class: {queries, node_visits, object_tests, tri_tests}}."""
        lib = hip_lib()
        n = len(self.WORK_CLASSES) * len(self.WORK_FIELDS)
        buf = (C.c_int64 * n)()
        _check(lib.rtx_last_work(self._s, buf, n), lib, "rtx_last_work")
        nf = len(self.WORK_FIELDS)
        return {c: {f: int(buf[i * nf + j]) for j, f in enumerate(self.WORK_FIELDS)}
                for i, c in enumerate(self.WORK_CLASSES)}

    def kernel_time(self):
        lib = hip_lib()
        ms = C.c_double()
        n = C.c_int()
        _check(lib.rtx_kernel_time(self._s, C.byref(ms), C.byref(n)), lib, "rtx_kernel_time")
        return ms.value, n.value

    def frame_status(self, raise_on_bad: bool = True):
        """Outcome of the device-buffer renders issued so far (rtx_frame_status):
        (first_bad, bad_frames), (-1, 0) when every frame came out right.
        Raises RtxError on a wrong frame unless raise_on_bad is False."""
        lib = hip_lib()
        fb, nb = C.c_int64(), C.c_int64()
        rc = lib.rtx_frame_status(self._s, C.byref(fb), C.byref(nb))
        if rc != 0 and (raise_on_bad or rc != RTX_ERR_FRAME):
            _check(rc, lib, "rtx_frame_status")
        return fb.value, nb.value

    def overlap_count(self):
        """(pipelined renders, renders) since the last call (rtx_overlap_count)."""
        lib = hip_lib()
        a, b = C.c_int64(), C.c_int64()
        _check(lib.rtx_overlap_count(self._s, C.byref(a), C.byref(b)), lib, "rtx_overlap_count")
        return a.value, b.value

    def frame_contexts(self):
        """How many frame contexts the last render rotated over (rtx_frame_contexts; 1: not pipelined)."""
        lib = hip_lib()
        n = C.c_int32()
        _check(lib.rtx_frame_contexts(self._s, C.byref(n)), lib, "rtx_frame_contexts")
        return n.value

    def close(self):
        if self._s:
            hip_lib().rtx_scene_destroy(self._s)
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_pixels(opts: RenderOptions, height: int, tile: int, shard: int, nshards: int, packed: bool) -> int:
    p = opts.params(height, tile, shard, nshards, packed)
    n = C.c_int64()
    hip_lib().rtx_shard_pixels(C.byref(p), C.byref(n))
    return n.value


def owned_tiles(width: int, height: int, tile: int, shard: int, nshards: int):
    """Tile ids (row-major from the bottom-left) a shard renders, in its packed
    order (rtx_shard_tiles: the deal of rtx_render.hip's deal_tile — deal
    index d = shard + k * nshards is tile row d // tx, column
    (d % tx + row) % tx, i.e. diagonal stripes)."""
    lib = host_lib()
    n = C.c_int32()
    _check_host(lib.rtx_shard_tiles(width, height, tile, shard, nshards, None, 0, C.byref(n)), "rtx_shard_tiles")
    ids = np.zeros(n.value, np.int32)
    _check_host(lib.rtx_shard_tiles(width, height, tile, shard, nshards, ids.ctypes.data, n.value, C.byref(n)),
                "rtx_shard_tiles")
    return [int(t) for t in ids]


def unpack_tiles(packed: np.ndarray, width: int, height: int, tile: int, shard: int, nshards: int,
                 out: np.ndarray, channels: int = 3):
    """Scatter a shard's packed tiles into a full (height, width, c) frame
    (rtx_unpack_tiles, the reassembly the multi-GPU driver runs)."""
    src = np.ascontiguousarray(packed)
    assert out.flags["C_CONTIGUOUS"] and out.dtype == src.dtype and out.shape[:2] == (height, width)
    elem = src.dtype.itemsize * channels
    _check_host(host_lib().rtx_unpack_tiles(src.ctypes.data, width, height, tile, shard, nshards, elem,
                                            out.ctypes.data), "rtx_unpack_tiles")
    return out


def read_image(path: str):
    """readImage (fileio/images.cc:47-53): (h, w, channels) uint8, row 0 = bottom."""
    lib = host_lib()
    w, h, ch = C.c_int32(), C.c_int32(), C.c_int32()
    _check_host(lib.rtx_read_image(path.encode(), C.byref(w), C.byref(h), C.byref(ch), None, 0), "rtx_read_image")
    out = np.zeros((h.value, w.value, ch.value), np.uint8)
    _check_host(lib.rtx_read_image(path.encode(), C.byref(w), C.byref(h), C.byref(ch), out.ctypes.data, out.size),
                "rtx_read_image")
    return out


def pack_tiles(full: np.ndarray, width: int, height: int, tile: int, shard: int, nshards: int) -> np.ndarray:
    """Gather a shard's tiles out of a full (height, width, c) frame into the
    packed layout the kernel writes with packed=1 (tile order, tile*tile
    pixels per tile, rows inside a tile from the bottom, zero padding)."""
    tx = (width + tile - 1) // tile
    tiles = owned_tiles(width, height, tile, shard, nshards)
    c = full.shape[2]
    out = np.zeros((len(tiles), tile, tile, c), full.dtype)
    for k, t in enumerate(tiles):
        x0, y0 = (t % tx) * tile, (t // tx) * tile
        w = min(tile, width - x0)
        h = min(tile, height - y0)
        out[k, :h, :w] = full[y0:y0 + h, x0:x0 + w]
    return out.reshape(-1)


def write_image(path: str, rgb8: np.ndarray):
    """writeImage (fileio/images.cc:59-68); rgb8 is (h, w, 3) with row 0 at the bottom."""
    a = np.ascontiguousarray(rgb8, dtype=np.uint8)
    h, w = a.shape[:2]
    rc = host_lib().rtx_write_image(path.encode(), w, h, a.ctypes.data)
    if rc != 0:
        raise RtxError(host_lib().rtx_host_last_error().decode())


def device_count() -> int:
    n = C.c_int()
    hip_lib().rtx_device_count(C.byref(n))
    return n.value
