#!/usr/bin/env python3
"""raycheck — render every .ray under a directory with two ray tracers and
compare the images, like the reference's grading harness
(ray/raycheck.py:82-116): `--exec` renders into out/image, `--ref` into
out/refcache (re-rendered when the reference binary's sha256 changes,
raycheck.py:57-80), both with `-r 5` plus `--flags`; PASS when the RMS over
the flattened RGB8 is below --maxrms (default 10.0, raycheck.py:20-33).

The reference computes the RMS on uint8 arrays, so `image - ref` wraps
modulo 256; both the wrapped figure (what the
reference prints) and the true one are reported.

--strict adds the north-star bar: both binaries also dump their float64
image (--dump-f64) and per-sample primary hit records (--dump-hits); PASS
needs |rgb diff| <= 1e-4 and object / face / BVH-leaf ids and ray counts
bit-exact.  Both binaries must understand those long options (bin/ray and
oracle/_build/ray_oracle do).

Typical use (GPU box): tools/raycheck.py --exec cs378hgraphics-raytracer_amd/bin/ray
    --ref oracle/_build/ray_oracle --scenes tests/golden/newScene --flags "-w 64" --strict
"""
import argparse
import hashlib
import os
import shutil
import struct
import subprocess
import sys
import zlib
from math import sqrt

import numpy as np

HIT_DTYPE = np.dtype([("object", "<i4"), ("face", "<i4"), ("scene_leaf", "<i4"), ("mesh_leaf", "<i4"),
                      ("nrays", "<i4"), ("pad", "<i4"), ("t", "<f8")])


# ------------------------------------------------------------------ image readers
def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def read_png(path):
    """8-bit RGB / RGBA, non-interlaced PNG -> uint8 (h, w, 3), first row = top."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError(f"{path}: not a PNG")
    pos, idat, w = 8, [], None
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        kind = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if kind == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
            if depth != 8 or ctype not in (2, 6) or interlace:
                raise ValueError(f"{path}: unsupported PNG (depth {depth}, colour type {ctype})")
            bpp = 3 if ctype == 2 else 4
        elif kind == b"IDAT":
            idat.append(body)
        elif kind == b"IEND":
            break
    raw = zlib.decompress(b"".join(idat))
    stride = w * bpp
    out = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    for r in range(h):
        ft = raw[r * (stride + 1)]
        line = np.frombuffer(raw, np.uint8, stride, r * (stride + 1) + 1).astype(np.int32)
        if ft == 0:
            cur = line
        elif ft == 2:
            cur = (line + prev) & 255
        else:  # sub / average / paeth depend on the reconstructed left byte
            cur = np.zeros(stride, np.int32)
            for x in range(stride):
                a = cur[x - bpp] if x >= bpp else 0
                b = prev[x]
                c = prev[x - bpp] if x >= bpp else 0
                pred = a if ft == 1 else ((a + b) >> 1 if ft == 3 else _paeth(a, b, c))
                cur[x] = (line[x] + pred) & 255
        out[r] = cur
        prev = cur
    return out.reshape(h, w, bpp)[:, :, :3]


def read_bmp(path):
    """24-bit BMP -> uint8 (h, w, 3), first row = top (as an image viewer shows it)."""
    with open(path, "rb") as f:
        data = f.read()
    off, = struct.unpack("<I", data[10:14])
    w, h = struct.unpack("<ii", data[18:26])
    bits, = struct.unpack("<H", data[28:30])
    if bits != 24:
        raise ValueError(f"{path}: {bits}-bit BMP unsupported")
    stride = (w * 3 + 3) & ~3
    rows = np.frombuffer(data, np.uint8, stride * abs(h), off).reshape(abs(h), stride)[:, :w * 3]
    img = rows.reshape(abs(h), w, 3)[:, :, ::-1]
    return img[::-1] if h > 0 else img


def read_image(path):
    with open(path, "rb") as f:
        magic = f.read(8)
    return read_png(path) if magic.startswith(b"\x89PNG") else read_bmp(path)


# ------------------------------------------------------------------ comparison
def rms(image, ref):
    """(wrapped, true) RMS over the flattened RGB8 (raycheck.py:20-33)."""
    a = image.reshape(-1)
    b = ref.reshape(-1)
    wrapped = (a - b).astype(np.float64)  # uint8 arithmetic wraps, as in the reference
    true = a.astype(np.float64) - b.astype(np.float64)
    return float(np.linalg.norm(wrapped) / sqrt(wrapped.size)), float(np.linalg.norm(true) / sqrt(true.size))


def strict_compare(f64_a, f64_b, hits_a, hits_b, tol=1e-4):
    """north-star bar: RGB within tol, hit ids / ray counts bit-exact."""
    a = np.fromfile(f64_a, np.float64)
    b = np.fromfile(f64_b, np.float64)
    if a.shape != b.shape:
        return False, f"f64 size {a.size} vs {b.size}"
    d = float(np.abs(a - b).max()) if a.size else 0.0
    ha = np.fromfile(hits_a, HIT_DTYPE)
    hb = np.fromfile(hits_b, HIT_DTYPE)
    if ha.shape != hb.shape:
        return False, f"hit records {ha.size} vs {hb.size}"
    bad = [f for f in ("object", "face", "scene_leaf", "mesh_leaf", "nrays") if not np.array_equal(ha[f], hb[f])]
    ok = d <= tol and not bad
    return ok, f"max|drgb| {d:.3g}" + (f", ids differ: {','.join(bad)}" if bad else ", ids bit-exact")


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 15), b""):
            h.update(chunk)
    return h.hexdigest()


def run(cmd, timeout=None, stdout=None, stderr=None):
    try:
        return subprocess.run(cmd, stdout=stdout, stderr=stderr, timeout=timeout).returncode
    except subprocess.TimeoutExpired:
        return 124


def raycheck(args):
    for d in (args.scenes,):
        if not os.path.isdir(d):
            print(f"{d} is not a directory")
            return 2
    for f in (args.exec, args.ref):
        if not os.path.isfile(f):
            print(f"{f} does not exist")
            return 2
    os.makedirs(args.out, exist_ok=True)
    refcache = os.path.join(args.out, "refcache")
    sig_path = os.path.join(refcache, "signature")
    sig = sha256(args.ref) + "|" + args.flags + ("|strict" if args.strict else "")
    if os.path.exists(sig_path) and open(sig_path).read() != sig:
        shutil.rmtree(refcache)
    os.makedirs(refcache, exist_ok=True)
    with open(sig_path, "w") as f:
        f.write(sig)
    flags = ["-r", "5"] + args.flags.split()
    n_pass = n_fail = 0
    for root, _dirs, files in os.walk(args.scenes):
        for fn in sorted(files):
            if not fn.endswith(".ray"):
                continue
            rayfn = os.path.join(root, fn)
            relbase = os.path.splitext(os.path.relpath(rayfn, args.scenes))[0]
            for sub in ("image", "refcache", "stdio"):
                os.makedirs(os.path.dirname(os.path.join(args.out, sub, relbase)), exist_ok=True)
            img = os.path.join(args.out, "image", relbase + ".png")
            ref = os.path.join(refcache, relbase + ".std.png")
            extra_e, extra_r = [], []
            if args.strict:
                extra_e = ["--dump-f64", img + ".f64", "--dump-hits", img + ".hits"]
                extra_r = ["--dump-f64", ref + ".f64", "--dump-hits", ref + ".hits"]
            if not os.path.exists(ref):
                run([args.ref] + flags + extra_r + [rayfn, ref])
            with open(os.path.join(args.out, "stdio", relbase + ".out"), "w") as so, \
                    open(os.path.join(args.out, "stdio", relbase + ".err"), "w") as se:
                rc = run([args.exec] + flags + extra_e + [rayfn, img], timeout=args.timelimit, stdout=so, stderr=se)
            if rc != 0 or not os.path.exists(img) or not os.path.exists(ref):
                both_failed = rc != 0 and not os.path.exists(ref)
                tag = "[PASS] " if both_failed else "[FAIL] "
                print(f"{tag}{relbase}: exec rc={rc}, ref image {'present' if os.path.exists(ref) else 'missing'}")
                n_pass += both_failed
                n_fail += not both_failed
                continue
            a, b = read_image(img), read_image(ref)
            if a.shape != b.shape:
                print(f"[FAIL] {relbase}: size {a.shape} vs {b.shape}")
                n_fail += 1
                continue
            wrapped, true = rms(a, b)
            ok = wrapped < args.maxrms
            msg = f"{relbase} RMS: {wrapped} (no wrap: {true})"
            if args.strict:
                sok, smsg = strict_compare(img + ".f64", ref + ".f64", img + ".hits", ref + ".hits")
                ok = ok and sok
                msg += "; strict: " + smsg
            print(("[PASS] " if ok else "[WARNING] ") + msg)
            n_pass += ok
            n_fail += not ok
    print(f"raycheck: {n_pass} passed, {n_fail} failed")
    return 0 if n_fail == 0 else 1


def main(argv=None):
    ap = argparse.ArgumentParser(description="Grading a ray tracer against a reference (raycheck.py)",
                                 formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument("--exec", metavar="RAY", default="cs378hgraphics-raytracer_amd/bin/ray")
    ap.add_argument("--ref", metavar="RAY.STD", default="oracle/_build/ray_oracle")
    ap.add_argument("--scenes", metavar="DIRECTORY", default="tests/golden/newScene")
    ap.add_argument("--out", metavar="DIRECTORY", default="raycheck.out")
    ap.add_argument("--timelimit", metavar="SECONDS", type=int, default=180)
    ap.add_argument("--maxrms", metavar="NUMBER", type=float, default=10.0)
    ap.add_argument("--flags", default="", help="extra flags for both binaries (e.g. '-w 64')")
    ap.add_argument("--strict", action="store_true", help="also require f64 within 1e-4 and bit-exact hit ids")
    return raycheck(ap.parse_args(argv))


if __name__ == "__main__":
    sys.exit(main())
