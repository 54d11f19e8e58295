#!/usr/bin/env python3
"""Next-hit queries per shadow walk (GPU box): renders a scene with stats
and prints the walk launches' query count against the shadow rays traced
(RtxStats / rtx_last_work).  Queries per walk > 1 are walk continuations
through transmissive hits, each a traversal from the root.
usage: python tools/walk_queries.py [SCENE.ray] [flags...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench

    pkg = bench.load_package()
    scene = sys.argv[1] if len(sys.argv) > 1 else "trimesh2_glass.ray"
    flags = sys.argv[2:] or "-w 480 -r 5 -O r -A 4".split()
    opts = pkg.RenderOptions.from_cli(flags)
    host = pkg.HostScene(os.path.join(ROOT, "scenes", scene))
    dev = pkg.DeviceScene(host, 0)
    st = dev.render(opts, want_f64=False, stats=True)["stats"]
    k = st["kernels"]
    print(json.dumps({"scene": scene, "flags": " ".join(flags), "shadow_traced": st["shadow_traced"],
                      "walk_queries": k["next"]["queries"], "closest_queries": k["closest"]["queries"],
                      "queries_per_walk": round(k["next"]["queries"] / max(1, st["shadow_traced"]), 3),
                      "next_node_visits_per_query": round(k["next"]["node_visits"] / max(1, k["next"]["queries"]), 1),
                      "tail": k["tail"]}))


if __name__ == "__main__":
    main()
