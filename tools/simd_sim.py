#!/usr/bin/env python3
"""CPU model of trace_kernel's wave stepping (tools/simd_sim.hip): how many
wave steps run the record / object / leaf code under a lane-selection
policy, for the headline frame's camera rays (closest-hit queries) and the
first shadow-walk queries from their hits (next-hit queries toward each
point light, bounded at half the light distance like the first walk query).

usage: python tools/simd_sim.py [--rows N] [--scene trimesh2.ray]
Costs per class are the VALU instruction counts of the code each runs
(rough, from the ISA; --cost REC OBJ LEAF to override)."""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SRC = os.path.join(ROOT, "tools", "simd_sim.hip")
LIB = os.path.join(ROOT, "tools", "_build", "libsimd_sim.so")


def build():
    deps = [SRC] + [os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "csrc", "hip", f)
                    for f in ("rtx_traverse.h", "rtx_device.h")]
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "--offload-host-only",
                        "-ffp-contract=off", "-fno-fast-math", "-I" + os.path.join(ROOT, "include"), "-shared",
                        "-o", LIB, SRC], check=True)
    return C.CDLL(LIB)


def camera_rays(pkg, host, width, rows, spp_side=4):
    d = host.desc
    cam = d.camera
    eye, look, u, v = (np.array(x[:3], np.float64) for x in (cam.eye, cam.look, cam.u, cam.v))
    h = host.height_for(width)
    s = spp_side
    ys = np.linspace(0, h - 1, rows).astype(int)
    P, D = [], []
    for j in ys:
        for i in range(width):  # pixel (i, j): its s*s samples, consecutive (4 pixels per wave)
            for k in range(s * s):
                pi, pj = i * s + k // s, j * s + k % s
                sx, sy = pi / (width * s), pj / (h * s)
                dd = look + (sx - 0.5) * u + (sy - 0.5) * v
                D.append(dd / np.sqrt(dd @ dd))
                P.append(eye)
    return np.array(P), np.array(D)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="trimesh2.ray")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--rows", type=int, default=6)
    ap.add_argument("--cost", type=float, nargs=3, default=[250.0, 300.0, 350.0])
    args = ap.parse_args()
    import bench

    pkg = bench.load_package()
    host = pkg.HostScene(os.path.join(ROOT, "scenes", args.scene))
    L = build()
    L.simd_sim_run.argtypes = [C.POINTER(pkg.RtxSceneDesc), C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                               C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]
    P, D = camera_rays(pkg, host, args.width, args.rows)
    n = len(P)
    # closest hits of the camera rays (the traversal harness of the tests)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_traverse_host as th

    TH = th._harness(pkg)
    t, o, f, nh, _ = th._run(TH, pkg, host, 1, P, D, np.full(n, 1e308), 1)
    hit = o[:, 0] >= 0
    Ph = P[hit] + t[hit, 0:1] * D[hit]
    nl = host.desc.n_lights  # RtxLight: 200 B = int32 type, pad, then 24 doubles (pos at 4..6)
    raw = bytes((C.c_char * (200 * nl)).from_address(host.desc.lights))
    SP, SD, SL = [], [], []
    for k in range(nl):
        if np.frombuffer(raw[k * 200:k * 200 + 4], np.int32)[0] != 1:  # point lights only
            continue
        lp = np.frombuffer(raw[k * 200 + 8:k * 200 + 200], np.float64)[3:6]
        dv = lp - Ph
        dist = np.sqrt((dv * dv).sum(1))
        SD.append(dv / dist[:, None])
        SP.append(Ph - 1e-8 * D[hit])
        SL.append(dist / 2 * (1 + 1e-6))
    # walk records are appended per wave of hits, light by light
    SP, SD, SL = np.concatenate(SP), np.concatenate(SD), np.concatenate(SL)
    out = np.zeros(8, np.int64)
    cost = np.array(args.cost)
    print(f"{n} camera rays, {len(SP)} first shadow queries; costs {cost.tolist()}")
    for name, q, PP, DD, TL in (("closest", 1, P, D, np.full(n, 1e308)), ("walk", 2, SP, SD, SL)):
        PP, DD, TL = (np.ascontiguousarray(x, np.float64) for x in (PP, DD, TL))
        for pol, k1, k2 in ((0, 16, 0), (0, 8, 0), (0, 32, 0), (0, 65, 0), (1, 16, 8), (1, 16, 16), (1, 16, 24),
                            (1, 8, 16), (2, 16, 8), (2, 16, 16), (2, 16, 32)):
            rc = L.simd_sim_run(C.byref(host.desc), q, len(PP), PP.ctypes.data, DD.ctypes.data, TL.ctypes.data,
                                pol, k1, k2, out.ctypes.data)
            assert rc == 0
            runs, lanes, ws = out[0:3], out[3:6], out[6]
            c = float((runs * cost).sum())
            print(f"{name:7s} policy {pol} k1={k1:2d} k2={k2:2d}: wave steps {ws:9d} runs rec/obj/leaf "
                  f"{runs[0]:9d} {runs[1]:9d} {runs[2]:9d}  lanes/run {lanes[0] / max(1, runs[0]):5.1f} "
                  f"{lanes[1] / max(1, runs[1]):5.1f} {lanes[2] / max(1, runs[2]):5.1f}  cost/query "
                  f"{c * 64 / out[7]:8.0f}")


if __name__ == "__main__":
    main()
