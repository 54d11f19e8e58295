#!/usr/bin/env python3
"""PNG fixtures for the texture reader (readPNG, pngimage.cpp:195-216).

Writes small PNGs of every colour type / bit depth / filter / interlace
combination the reference's libpng transforms cover into
tests/golden/feature/, plus png_expected.npz: the pixels each file must
decode to after those transforms (palette and low-depth gray expanded,
tRNS -> alpha, 16 -> 8 bits by the high byte, gray -> RGB, gamma only with a
gAMA chunk), rows flipped so row 0 is the picture's bottom.  The expected
arrays are computed here from the pixel values this script chose, not by
decoding, so they pin rtx_read_image independently.  The gamma case follows
libpng 1.6's published 8-bit table rule (no libpng here: parity of that one
case vs libpng itself is unpinned).  Deterministic (seed 5).
"""
import math
import os
import struct
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "feature")


def chunk(t, data):
    c = struct.pack(">I", len(data)) + t + data
    return c + struct.pack(">I", zlib.crc32(t + data) & 0xffffffff)


def paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def filter_rows(rows, bpp, first_filter):
    """rows: list of bytes (packed samples); filter type cycles 0..4."""
    out = bytearray()
    prev = bytes(len(rows[0])) if rows else b""
    for y, row in enumerate(rows):
        ft = (first_filter + y) % 5
        out.append(ft)
        for x in range(len(row)):
            a = row[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            pred = [0, a, b, (a + b) // 2, paeth(a, b, c)][ft]
            out.append((row[x] - pred) & 0xff)
        prev = row
    return bytes(out)


def pack_row(samples, depth):
    """samples: 1-D ints of one row (all channels interleaved)."""
    if depth == 16:
        return b"".join(struct.pack(">H", int(v)) for v in samples)
    if depth == 8:
        return bytes(int(v) for v in samples)
    out, acc, nb = bytearray(), 0, 0
    for v in samples:
        acc = (acc << depth) | int(v)
        nb += depth
        if nb == 8:
            out.append(acc)
            acc, nb = 0, 0
    if nb:
        out.append(acc << (8 - nb))
    return bytes(out)


ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def write_png(path, img, ctype, depth, interlace=False, plte=None, trns=None, gama=None):
    """img: (h, w, spp) native sample values."""
    h, w, spp = img.shape
    bpp = max(1, spp * depth // 8)
    data = b""
    passes = ADAM7 if interlace else [(0, 0, 1, 1)]
    for k, (x0, y0, dx, dy) in enumerate(passes):
        sub = img[y0::dy, x0::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        rows = [pack_row(sub[y].reshape(-1), depth) for y in range(sub.shape[0])]
        data += filter_rows(rows, bpp, k)
    out = b"\x89PNG\r\n\x1a\n"
    out += chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 1 if interlace else 0))
    if gama is not None:
        out += chunk(b"gAMA", struct.pack(">I", gama))
    if plte is not None:
        out += chunk(b"PLTE", bytes(np.asarray(plte, np.uint8).reshape(-1)))
    if trns is not None:
        out += chunk(b"tRNS", bytes(trns))
    z = zlib.compress(data, 9)
    # split IDAT in two chunks (readers must concatenate)
    out += chunk(b"IDAT", z[: len(z) // 2]) + chunk(b"IDAT", z[len(z) // 2:])
    out += chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(out)


def flip(a):
    return np.ascontiguousarray(a[::-1])


def gamma_table(gama):
    corr = math.floor(1e15 / gama / 220000.0 + 0.5)
    if 95000 <= corr <= 105000:
        return np.arange(256)
    t = np.arange(256)
    for v in range(1, 255):
        t[v] = math.floor(255 * math.pow(v / 255.0, corr * 0.00001) + 0.5)
    return t


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(5)
    exp = {}
    # 1. 8-bit RGB, all five filters
    a = rng.integers(0, 256, (9, 13, 3))
    write_png(os.path.join(OUT, "png_rgb8.png"), a, 2, 8)
    exp["png_rgb8"] = flip(a.astype(np.uint8))
    # 2. 4-bit palette with tRNS -> RGBA
    pal = rng.integers(0, 256, (16, 3))
    idx = rng.integers(0, 16, (7, 10, 1))
    trns = [255, 0, 128, 7]
    write_png(os.path.join(OUT, "png_pal4.png"), idx, 3, 4, plte=pal, trns=trns)
    alpha = np.array([trns[i] if i < len(trns) else 255 for i in range(16)])
    e = np.concatenate([pal[idx[..., 0]], alpha[idx[..., 0]][..., None]], axis=2)
    exp["png_pal4"] = flip(e.astype(np.uint8))
    # 3. 16-bit gray -> RGB, high byte
    g = rng.integers(0, 65536, (5, 6, 1))
    write_png(os.path.join(OUT, "png_gray16.png"), g, 0, 16)
    hb = (g[..., 0] >> 8)
    exp["png_gray16"] = flip(np.stack([hb, hb, hb], axis=2).astype(np.uint8))
    # 4. 2-bit gray -> 8 bits (x 85) -> RGB
    g2 = rng.integers(0, 4, (6, 7, 1))
    write_png(os.path.join(OUT, "png_gray2.png"), g2, 0, 2)
    v = g2[..., 0] * 85
    exp["png_gray2"] = flip(np.stack([v, v, v], axis=2).astype(np.uint8))
    # 5. RGBA 8-bit, Adam7 interlaced
    r = rng.integers(0, 256, (10, 11, 4))
    write_png(os.path.join(OUT, "png_rgba_adam7.png"), r, 6, 8, interlace=True)
    exp["png_rgba_adam7"] = flip(r.astype(np.uint8))
    # 6. 16-bit RGB with tRNS colour key -> RGBA
    c16 = rng.integers(0, 65536, (4, 5, 3))
    key = c16[1, 2].copy()
    write_png(os.path.join(OUT, "png_rgb16_trns.png"), c16, 2, 16,
              trns=list(struct.pack(">HHH", *[int(x) for x in key])))
    al = np.where(np.all(c16 == key, axis=2), 0, 255)
    exp["png_rgb16_trns"] = flip(np.concatenate([c16 >> 8, al[..., None]], axis=2).astype(np.uint8))
    # 7. gray + alpha 8-bit -> RGBA
    ga = rng.integers(0, 256, (3, 4, 2))
    write_png(os.path.join(OUT, "png_graya8.png"), ga, 4, 8)
    exp["png_graya8"] = flip(np.stack([ga[..., 0]] * 3 + [ga[..., 1]], axis=2).astype(np.uint8))
    # 8. gAMA 1.0 (linear file): libpng applies 1 / 2.2
    lg = rng.integers(0, 256, (4, 6, 3))
    write_png(os.path.join(OUT, "png_gamma_linear.png"), lg, 2, 8, gama=100000)
    exp["png_gamma_linear"] = flip(gamma_table(100000)[lg].astype(np.uint8))
    # 9. gAMA 1/2.2 (sRGB-like): insignificant correction, values unchanged
    write_png(os.path.join(OUT, "png_gamma_srgb.png"), lg, 2, 8, gama=45455)
    exp["png_gamma_srgb"] = flip(lg.astype(np.uint8))
    # 10. the scene textures (tests/golden/feature/png_tex.ray): a 48x40
    # RGB diffuse map (palette-free, filtered) and a gray bump map
    yy, xx = np.mgrid[0:40, 0:48]
    tex = np.stack([(xx * 5) % 256, (yy * 6) % 256, ((xx + yy) * 3) % 256], axis=2)
    tex[(xx // 8 + yy // 8) % 2 == 0] //= 2
    write_png(os.path.join(OUT, "png_tex_diffuse.png"), tex, 2, 8)
    exp["png_tex_diffuse"] = flip(tex.astype(np.uint8))
    bump = (128 + 100 * np.sin(xx / 3.0) * np.cos(yy / 4.0)).astype(int)
    write_png(os.path.join(OUT, "png_tex_bump.png"), bump[..., None], 0, 8)
    exp["png_tex_bump"] = flip(np.stack([bump] * 3, axis=2).astype(np.uint8))
    np.savez_compressed(os.path.join(OUT, "png_expected.npz"), **exp)
    print("wrote", len(exp), "PNG fixtures to", OUT)


if __name__ == "__main__":
    sys.exit(main())
