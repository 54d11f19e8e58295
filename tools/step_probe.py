#!/usr/bin/env python3
"""Per-launch step statistics of one shard (or the full frame): renders with
the counting kernels under RTX_DEBUG=2, so every closest-hit launch prints its
duration, the most steps any of its queries took and how many took > 100
(rtx_render.hip, trace_kernel STATS).  ms / max steps ~ the time of one step
of the wave that finishes last.
usage (GPU box): RTX_DEBUG=2 python tools/step_probe.py [--flags "..."] [--scene S] RANK N"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench

    pkg = bench.load_package()
    args = sys.argv[1:]
    flags, scene = "-w 1920 -r 5 -O r -A 4", "trimesh2.ray"
    while args and args[0] in ("--flags", "--scene"):
        if args[0] == "--flags":
            flags = args[1]
        else:
            scene = args[1]
        args = args[2:]
    rank, n = (int(args[0]), int(args[1])) if len(args) >= 2 else (0, 1)
    opts = pkg.RenderOptions.from_cli(flags.split())
    dev = pkg.DeviceScene(pkg.HostScene(os.path.join(ROOT, "scenes", scene)), 0)
    tile = 16 if n > 1 else 0
    out = dev.render(opts, want_f64=False, stats=True, tile=tile, shard=rank, nshards=n, packed=n > 1)
    print({k: v for k, v in out["stats"].items() if k != "kernels"}, flush=True)


if __name__ == "__main__":
    main()
