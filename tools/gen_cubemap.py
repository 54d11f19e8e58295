#!/usr/bin/env python3
"""Write the six-face cube-map fixture tests/golden/cubemap/{pos,neg}{x,y,z}.bmp
(deterministic gradients + a checker per face, 32x24 so bilinear filtering and
the non-square case are exercised).  The reference ships no cube-map images;
names follow what TraceUI::matchCubemapFiles matches (ui/TraceUI.cc:87-146).
The directory must hold exactly these six files: the matcher's
find_first_of would claim other names too."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402

FACES = ["posx", "negx", "posy", "negy", "posz", "negz"]
BASE = [(230, 60, 40), (40, 200, 70), (50, 90, 240), (240, 220, 40), (200, 60, 220), (40, 220, 220)]


def main():
    pkg = load_package()
    out = os.path.join(ROOT, "tests", "golden", "cubemap")
    os.makedirs(out, exist_ok=True)
    w, h = 32, 24
    y, x = np.mgrid[0:h, 0:w]
    for k, (name, base) in enumerate(zip(FACES, BASE)):
        img = np.zeros((h, w, 3), np.float64)
        for c in range(3):
            img[..., c] = base[c] * (0.35 + 0.65 * x / (w - 1)) * (0.5 + 0.5 * y / (h - 1))
        img[((x // 4 + y // 4 + k) % 2) == 0] *= 0.6
        rgb = np.ascontiguousarray(np.clip(img, 0, 255).astype(np.uint8))
        rc = pkg.host_lib().rtx_write_image(os.path.join(out, name + ".bmp").encode(), w, h, rgb.ctypes.data)
        assert rc == 0


if __name__ == "__main__":
    main()
