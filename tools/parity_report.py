#!/usr/bin/env python3
"""Print a parity report (GPU vs CPU restatement) for every case in
tests/cases.py: max |rgb diff|, hit coverage, ray counts, timings.  Runs on a
GPU box; writes JSON to stdout (or --out)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package, load_oracle, scene_path  # noqa: E402
from cases import CASES  # noqa: E402

import numpy as np  # noqa: E402


def main():
    pkg = load_package()
    orc = load_oracle()
    rows = []
    for name, scene, flags in CASES:
        path = scene_path(scene)
        opts = pkg.RenderOptions.from_cli(flags.split())
        dev = pkg.DeviceScene(pkg.HostScene(path), 0)
        t0 = time.time()
        g = dev.render(opts, want_f64=True, want_hits=True, stats=True)
        tg = time.time() - t0
        t0 = time.time()
        r = orc.render(pkg, path, opts, want_hits=True)
        tr = time.time() - t0
        d = np.abs(g["rgb"] - r["rgb"])
        row = {
            "case": name, "flags": flags, "max_abs_rgb": float(d.max()), "mean_rgb": float(r["rgb"].mean()),
            "rgb8_equal_frac": float((g["rgb8"] == r["rgb8"]).mean()),
            "hit_frac": float((r["hits"]["object"] >= 0).mean()),
            "ids_equal": bool(all(np.array_equal(g["hits"][f], r["hits"][f])
                                  for f in ("object", "face", "scene_leaf", "mesh_leaf", "nrays"))),
            "gpu_rays": g["stats"]["rays"], "cpu_rays": r["stats"]["rays"],
            "gpu_kernel_ms": g["stats"]["kernel_ms"], "gpu_wall_s": tg, "cpu_wall_s": tr,
            "gpu_node_visits": g["stats"]["node_visits"], "cpu_node_visits": r["stats"]["node_visits"],
            "gpu_tri_tests": g["stats"]["tri_tests"], "cpu_tri_tests": r["stats"]["tri_tests"],
        }
        rows.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
