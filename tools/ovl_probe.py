#!/usr/bin/env python3
"""Time one -O o (overlapping media) render on the GPU and its ray counts.
usage (GPU box): python tools/ovl_probe.py WIDTH [SCENE] [DEPTH]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package, scene_path  # noqa: E402

pkg = load_package()
w = sys.argv[1]
scene = sys.argv[2] if len(sys.argv) > 2 else "spheres_overlap.ray"
depth = sys.argv[3] if len(sys.argv) > 3 else "5"
opts = pkg.RenderOptions.from_cli(f"-w {w} -r {depth} -O o".split())
host = pkg.HostScene(scene_path(scene))
dev = pkg.DeviceScene(host, 0)
t0 = time.time()
r = dev.render(opts, want_f64=True, stats=True)
print("gpu", scene, w, round(time.time() - t0, 3), "s", r["stats"], flush=True)
