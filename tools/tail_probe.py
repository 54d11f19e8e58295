#!/usr/bin/env python3
"""Critical-path probe (RTX_DEBUG=1 on the GPU box): render shard 0 of N of
the headline frame with stats and print the slowest tail chain."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

pkg = bench.load_package()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
shard = int(sys.argv[2]) if len(sys.argv) > 2 else 0
opts = pkg.RenderOptions.from_cli("-w 1920 -r 5 -O r -A 4".split())
host = pkg.HostScene(os.path.join(ROOT, "scenes", "trimesh2.ray"))
dev = pkg.DeviceScene(host, 0)
st = dev.render(opts, want_f64=False, stats=True, tile=32 if n > 1 else 0, shard=shard, nshards=n, packed=n > 1)["stats"]
print("shard", shard, "of", n, "stats-pass ms", round(st["kernel_ms"], 2), "rays", st["rays"])
