#!/usr/bin/env python3
"""Which camera rays of a frame make the long traversal queries: runs the
device traversal compiled for the host (tests/native/traverse_host.hip) on
one camera ray per pixel (pixel centres of sample 0) and prints the costliest
pixels, their hit objects, and a per-column / per-row histogram of the cost.
usage: python tools/ray_cost_probe.py [scene] [width] [height]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import bench
    from test_traverse_host import _harness
    pkg = bench.load_package()
    scene = sys.argv[1] if len(sys.argv) > 1 else "trimesh2.ray"
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 480
    host = pkg.HostScene(os.path.join(ROOT, "scenes", scene))
    h = int(sys.argv[3]) if len(sys.argv) > 3 else host.height_for(w)
    L = _harness(pkg)
    L.trav_host_cost.argtypes = [C.POINTER(pkg.RtxSceneDesc), C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_void_p]
    cam = host.desc.camera
    eye, look, u, v = (np.array(x[:]) for x in (cam.eye, cam.look, cam.u, cam.v))
    jj, ii = np.mgrid[0:h, 0:w]
    off = float(os.environ.get("PROBE_OFF", "0.5"))  # 0.5: pixel centres; 0: AA sample (0, 0)
    x = (ii.ravel() + off) / w - 0.5
    y = (jj.ravel() + off) / h - 0.5
    d = look[None] + x[:, None] * u[None] + y[:, None] * v[None]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    n = d.shape[0]
    P = np.ascontiguousarray(np.repeat(eye[None], n, 0))
    D = np.ascontiguousarray(d)
    nodes = np.zeros(n, np.int64)
    objs = np.zeros(n, np.int64)
    tris = np.zeros(n, np.int64)
    obj = np.zeros(n, np.int32)
    rc = L.trav_host_cost(C.byref(host.desc), n, P.ctypes.data, D.ctypes.data, nodes.ctypes.data, objs.ctypes.data,
                          tris.ctypes.data, obj.ctypes.data)
    assert rc == 0
    steps = nodes // 4 + objs + tris // 2  # rough step count (records, objects, leaves)
    order = np.argsort(-steps)
    print(f"{scene} {w}x{h}: mean cost {steps.mean():.1f}, p99 {np.percentile(steps, 99):.0f}, max {steps.max()}")
    for k in order[:25]:
        print(f"  px ({ii.ravel()[k]:4d},{jj.ravel()[k]:4d}) nodes {nodes[k]:6d} objs {objs[k]:4d} tris {tris[k]:6d} "
              f"hit object {obj[k]}")
    big = steps > 200
    print("costly rays (>200):", int(big.sum()), "by hit object:",
          {int(o): int(c) for o, c in zip(*np.unique(obj[big], return_counts=True))})
    cols = np.bincount(ii.ravel()[big], minlength=w)
    rows = np.bincount(jj.ravel()[big], minlength=h)
    print("columns with costly rays:", np.nonzero(cols)[0][:60].tolist())
    print("rows with costly rays:", np.nonzero(rows)[0][:60].tolist())


if __name__ == "__main__":
    main()
