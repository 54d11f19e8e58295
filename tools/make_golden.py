#!/usr/bin/env python3
"""Generate tests/golden/oracle_*.npz: small renders of the bundled fixtures
and stand-ins by the CPU restatement (oracle/).  These pin the oracle against
regressions (tests/test_golden.py) and give the GPU tests a fixed target.
They are NOT outputs of the original binary (unbuildable here; parity vs the
original is unpinned)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import cli_opts, load_package, load_oracle, scene_path  # noqa: E402

GOLDEN_CASES = [
    ("spheres_overlap", "spheres_overlap.ray", "-w 24 -r 5"),
    ("distance", "distance.ray", "-w 24 -r 3"),
    ("concrete_3", "concrete_3.ray", "-w 24 -r 5"),
    ("spotlight", "box_cyl_opaque_shadow_spotlight.ray", "-w 24 -r 2"),
    ("lava_box", "lava_box.ray", "-w 20 -r 3"),
    ("hitchcock", "hitchcock.ray", "-w 24 -r 3 -O r -A 2"),
    ("trimesh2_square", "trimesh2_square.ray", "-w 20 -r 5"),
    ("cones", "cones.ray", "-w 24 -r 4"),
    ("cubemap_cones", "cones.ray", "-w 24 -r 3 -c cubemap/posx.bmp"),
    ("overlap_spheres", "spheres_overlap.ray", "-w 24 -r 5 -O o"),
]


def main():
    pkg = load_package()
    orc = load_oracle()
    out = os.path.join(ROOT, "tests", "golden")
    only = set(sys.argv[1:])  # names to (re)generate; default all
    for name, scene, flags in GOLDEN_CASES:
        if only and name not in only:
            continue
        opts = cli_opts(pkg, flags)
        r = orc.render(pkg, scene_path(scene), opts, want_hits=True)
        np.savez_compressed(os.path.join(out, f"oracle_{name}.npz"), rgb=r["rgb"], rgb8=r["rgb8"],
                            hits=r["hits"], flags=np.array(flags), scene=np.array(scene),
                            rays=np.array(r["stats"]["rays"]))
        print(name, r["stats"]["rays"], float(r["rgb"].mean()))


if __name__ == "__main__":
    main()
