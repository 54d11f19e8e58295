"""The float record test (box_cons32, rtx_device.h; DESIGN.md "Float record
tests") never rejects a box that contains a point of the ray at t >= 0: the
requirement for the device's own BVH records, whose boxes only steer the walk
(the exact tests decide candidacy: objects' world boxes and leaf_ok).

Checked against an exact rational slab (fractions.Fraction) on adversarial
(ray, box) pairs: boxes that just touch the ray (the ray passes through a
face or an edge of the box, within a few ulps), rays with zero direction
components (the inside test: the box must be hit iff o lies in the slab),
large origins (the float rounding of o dominates), and near-parallel rays.
Runs the device code compiled for the host (tests/native/traverse_host.hip)."""
import ctypes as C
from fractions import Fraction as Fr

import numpy as np

from test_traverse_host import _harness


def exact_hit(o, d, lo, hi):
    """Does the ray o + t d, t >= 0, meet the closed box [lo, hi]?  Exact."""
    tmin, tmax = Fr(0), None
    for a in range(3):
        oa, da, la, ha = Fr(o[a]), Fr(d[a]), Fr(lo[a]), Fr(hi[a])
        if da == 0:
            if oa < la or oa > ha:
                return False
            continue
        t1, t2 = (la - oa) / da, (ha - oa) / da
        if t1 > t2:
            t1, t2 = t2, t1
        tmin = max(tmin, t1)
        tmax = t2 if tmax is None else min(tmax, t2)
        if tmin > tmax:
            return False
    return True


def _cases(rng, n):
    P, D, B = [], [], []
    for k in range(n):
        kind = k % 5
        scale = [1.0, 1e3, 1e6, 0.01, 50.0][k % 5]
        o = rng.normal(size=3) * scale
        d = rng.normal(size=3)
        if kind == 1:  # zero components
            d[rng.integers(0, 3)] = 0.0
            if k % 2:
                d[rng.integers(0, 3)] = 0.0
        if kind == 2:  # near-parallel to an axis plane
            d[rng.integers(0, 3)] *= 1e-9
        if abs(d).max() == 0.0:
            d[0] = 1.0
        d /= np.linalg.norm(d)
        # a point on the ray (or just off it), a box with a face through it
        t = abs(rng.normal()) * scale + 1e-3
        x = o + t * d
        ext = abs(rng.normal(size=3)) * scale * 0.1 + 1e-9
        lo, hi = x - ext * rng.random(3), x + ext * rng.random(3)
        ax = rng.integers(0, 3)
        eps = rng.choice([0.0, 1e-16, -1e-16, 1e-13, -1e-13, 1e-9, -1e-9]) * max(abs(x[ax]), 1.0)
        if rng.random() < 0.5:
            lo[ax] = x[ax] + eps  # the ray grazes the box's lower face
        else:
            hi[ax] = x[ax] + eps
        if kind == 1:  # zero axes: origin exactly on / just off the slab boundary
            za = np.nonzero(d == 0.0)[0]
            for a in za:
                lo[a] = o[a] + rng.choice([0.0, 1e-15, -1e-15]) * max(abs(o[a]), 1.0)
                hi[a] = max(hi[a], lo[a])
        lo, hi = np.minimum(lo, hi), np.maximum(lo, hi)
        P.append(o)
        D.append(d)
        B.append(np.concatenate([lo, hi]))
    return np.array(P), np.array(D), np.array(B)


def test_float_record_test_is_conservative(pkg):
    L = _harness(pkg)
    L.rec_test_host.argtypes = [C.c_int32] + [C.c_void_p] * 5
    rng = np.random.default_rng(2024)
    n = 6000
    P, D, B = _cases(rng, n)
    ok = np.zeros(n, np.int32)
    a = np.zeros(n, np.float32)
    assert L.rec_test_host(n, P.ctypes.data, D.ctypes.data, B.ctypes.data, ok.ctypes.data, a.ctypes.data) == 0
    hits = 0
    for k in range(n):
        if exact_hit(P[k], D[k], B[k, :3], B[k, 3:]):
            hits += 1
            assert ok[k] == 1, f"case {k}: exact hit rejected (o={P[k]!r}, d={D[k]!r}, box={B[k]!r})"
    assert hits > n // 3  # the cases really sit on the boundary of hitting
    # and the float test still culls: boxes clearly off the ray are rejected
    far = B.copy()
    far[:, :3] += 10.0 * (abs(B[:, 3:] - B[:, :3]).max(axis=1, keepdims=True) + 1.0) * np.sign(D + 1e-300) * -1
    far[:, 3:] = far[:, :3] + (B[:, 3:] - B[:, :3])
    ok2 = np.zeros(n, np.int32)
    assert L.rec_test_host(n, P.ctypes.data, D.ctypes.data, far.ctypes.data, ok2.ctypes.data, a.ctypes.data) == 0
    culled = sum(1 for k in range(n) if not exact_hit(P[k], D[k], far[k, :3], far[k, 3:]) and ok2[k] == 0)
    missed = sum(1 for k in range(n) if not exact_hit(P[k], D[k], far[k, :3], far[k, 3:]))
    assert missed > 0 and culled >= 0.9 * missed


def test_tiny_direction_components(pkg):
    """A nonzero direction component too small for a float reciprocal
    (|d| < 3.4e-39): the hit points drift off the origin's coordinate by
    t |d|, so that axis must not be an inside test.  Boxes that
    hold a far point of such a ray, but not the origin's coordinate on that
    axis, must pass."""
    L = _harness(pkg)
    L.rec_test_host.argtypes = [C.c_int32] + [C.c_void_p] * 5
    P, D, B = [], [], []
    for tiny in (1e-40, -2e-39, 3e-39, 5e-45, -1e-42):
        for ax in range(3):
            for t in (1e9, 1e12, 1e15):
                o = np.zeros(3)
                d = np.ones(3)
                d[ax] = tiny
                d[(ax + 1) % 3] = 0.0  # one zero axis too (an inside test that does hold)
                x = o + t * d
                lo, hi = x - abs(x) * 1e-3 - 1e-300, x + abs(x) * 1e-3 + 1e-300
                P.append(o)
                D.append(d)
                B.append(np.concatenate([lo, hi]))
    P, D, B = np.array(P), np.array(D), np.array(B)
    n = len(P)
    ok = np.zeros(n, np.int32)
    a = np.zeros(n, np.float32)
    assert L.rec_test_host(n, P.ctypes.data, D.ctypes.data, B.ctypes.data, ok.ctypes.data, a.ctypes.data) == 0
    for k in range(n):
        assert exact_hit(P[k], D[k], B[k, :3], B[k, 3:]), k
        assert ok[k] == 1, f"case {k}: exact hit rejected (d={D[k]!r}, box={B[k]!r})"


def test_prune_bounds_widen(pkg):
    """The record walk prunes a record entry whose float slab starts past the
    query's best t (or ends before its lower bound) against float copies of
    those bounds (visit4: f_up_wide / f_down_wide, rtx_device.h).  They must
    never be tighter than the doubles — up >= x >= dn exactly — over the
    whole double range: float-range edges, denormals, zeros, infinities."""
    L = _harness(pkg)
    L.prune_bounds_host.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(11)
    mant = rng.random(200000) + 1.0
    expo = rng.integers(-160, 140, 200000).astype(np.float64)
    x = np.concatenate([
        mant * np.exp2(expo) * np.where(rng.random(200000) < 0.5, -1.0, 1.0),
        rng.normal(size=20000) * 100.0,
        np.nextafter(np.float32(rng.normal(size=2000)).astype(np.float64), np.inf),  # just past a float
        np.nextafter(np.float32(rng.normal(size=2000)).astype(np.float64), -np.inf),
        np.array([0.0, -0.0, 1e-320, -1e-320, 1e-45, -1e-45, 1.2e-38, -1.2e-38, 3.4028234e38, -3.4028234e38,
                  3.5e38, -3.5e38, 1e308, -1e308, np.inf, -np.inf, 1e-5, 0.1, 1.0, 4096.0]),
    ])
    up = np.zeros(x.size, np.float32)
    dn = np.zeros(x.size, np.float32)
    assert L.prune_bounds_host(x.size, x.ctypes.data, up.ctypes.data, dn.ctypes.data) == 0
    assert np.all(up.astype(np.float64) >= x), x[up.astype(np.float64) < x][:5]
    assert np.all(dn.astype(np.float64) <= x), x[dn.astype(np.float64) > x][:5]
    # and not much wider than the tightest floats (a few ulps) where finite
    fin = np.isfinite(up) & (np.abs(x) > 1e-30) & (np.abs(x) < 1e38)
    rel = (up[fin].astype(np.float64) - x[fin]) / np.abs(x[fin])
    assert rel.max() < 2.0 ** -20
