#!/usr/bin/env python3
"""Time every BASELINE.json configuration once on one GPU (after one warmup
frame) and print one JSON line per config: frame ms, rays, Mrays/s.

Configs (BASELINE.json "configs"):
  C1 hitchcock 256x256 -r 1                 (the reference's CPU-scale case)
  C2 hitchcock 512x512 -r 3 -O r -A 2
  C3 trimesh2 1024x1024 -r 5 -O r -A 4      (square-aspect stand-in)
  C4 trimesh2 1920x1080 -r 5 DoF fd 2.5, 16 rays, aperture 0.05
  C5 dragon (1M triangles) 3840x2160 -r 5 -O a -A 8
  R1 trimesh2_glass 1920x1080 -r 5 -O r -A 4 (recursion-heavy: the headline
     geometry with reflective / transmissive materials; not a BASELINE config)
  A1 lava_box (rect area light) 1920 wide -r 5 -O s -A 4 (soft shadows, 4 picks)
  A2 box_cyl_opaque_shadow_spotlight (spot light) 1920 wide -r 5
The headline (trimesh2 1920x1080 -r 5 -O r -A 4) is bench.py's.
usage: python tools/bench_configs.py [C1 C2 ...]  (on the GPU box)
"""
import json
import os

# frame contexts: 2 x 3 slot-group streams want their own hardware queues; the
# environment may hold HIP's default of 4 (the GPU box does), so raise it
import sys  # (before the queue override below)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:
    if os.environ.get("GPU_MAX_HW_QUEUES"):
        print(f"{os.path.basename(__file__)}: GPU_MAX_HW_QUEUES={os.environ['GPU_MAX_HW_QUEUES']} raised to 16",
              file=sys.stderr)
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "C1": ("hitchcock.ray", "-w 256 -r 1"),
    "C2": ("hitchcock.ray", "-w 512 -r 3 -O r -A 2"),
    "C3": ("trimesh2_square.ray", "-w 1024 -r 5 -O r -A 4"),
    "C4": ("trimesh2.ray", "-w 1920 -r 5 -O d -A 2.5 -B 16 -C 0.05"),
    "C5": ("dragon.ray", "-w 3840 -r 5 -O a -A 8"),
    "R1": ("trimesh2_glass.ray", "-w 1920 -r 5 -O r -A 4"),
    # area / spot lights on the fused walks: the bundled
    # fixtures (ray/newScene) at 1920 wide, their own aspect ratios
    "A1": ("../tests/golden/newScene/lava_box.ray", "-w 1920 -r 5 -O s -A 4"),
    "A2": ("../tests/golden/newScene/box_cyl_opaque_shadow_spotlight.ray", "-w 1920 -r 5"),
}


def main():
    import bench

    names = sys.argv[1:] or list(CONFIGS)
    scenes = os.path.join(ROOT, "scenes")
    if "C5" in names and not os.path.exists(os.path.join(scenes, "dragon.ray")):
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_scenes.py"), "--dragon"], check=True,
                       stdout=subprocess.DEVNULL)
    pkg = bench.load_package()
    for name in names:
        scene, flags = CONFIGS[name]
        t0 = time.time()
        host = pkg.HostScene(os.path.join(scenes, scene))
        t_load = time.time() - t0
        t0 = time.time()
        dev = pkg.DeviceScene(host, 0)
        t_up = time.time() - t0
        opts = pkg.RenderOptions.from_cli(flags.split())
        st = dev.render(opts, want_f64=False, stats=True)["stats"]  # counting pass (also warms up)
        h = host.height_for(opts.width)
        dev.render(opts, want_f64=False)  # the timed kernels' first launch (code-object load) untimed
        walls = []
        for _ in range(3):
            t0 = time.time()
            dev.render(opts, want_f64=False)
            walls.append(time.time() - t0)
        wall = sorted(walls)[1]  # median of 3 (host-synchronous renders: wall clock)
        line = {"config": name, "scene": os.path.basename(scene), "flags": flags, "width": opts.width, "height": h,
                "triangles": host.info.n_faces, "load_s": round(t_load, 2), "upload_and_trees_s": round(t_up, 2),
                "frame_ms": round(wall * 1e3, 2), "rays": st["rays"],
                "mrays_per_s": round(st["rays"] / wall / 1e6, 2),
                "work": {k: st[k] for k in ("camera_rays", "secondary_rays", "shadow_rays", "node_visits",
                                            "object_tests", "tri_tests")},
                "fused_walks": os.environ.get("RTX_FUSE", "1") != "0" and os.environ.get("RTX_FUSE_AREA", "1") != "0",
                "path": ("megakernel" if os.environ.get("RTX_MEGAKERNEL", "0") not in ("", "0") else
                         "wavefront (adaptive levels)" if opts.aa_mode == pkg.RTX_AA_ADAPTIVE else "wavefront")}
        print(json.dumps(line), flush=True)
        dev.close()
        host.close()


if __name__ == "__main__":
    main()
