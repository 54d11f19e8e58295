"""The product's vector math (csrc/common/rt_math.h — host loader and gfx950
kernels) against the oracle's own restatement of glm 0.9.8.4
(oracle/glm_restated.h), bit for bit, on random and edge inputs.

The reference does every vector operation through glm 0.9.8.4 (pinned at
ray/cmake/glm.cmake:11,15; not vendored, not available offline).  The oracle
no longer includes the product's header, so a slip in
the product's operation order (dot's pairing, normalize's reciprocal, the
mat4 * vec4 column sums) shows up here and in the parity suite instead of
being shared by checker and product.  Call sites: RayTracer.cpp:77,149,162,
scene.h:57-62, light.cpp:21-73, material.cpp:34-69, camera.cpp:21-31,
RayTracer.cpp:388-394 (setPixel).

The two headers are compiled in separate translation units
(tests/native/math_pair_{product,oracle}.cpp) into one test library."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

NATIVE = [os.path.join(ROOT, "tests", "native", f) for f in ("math_pair_product.cpp", "math_pair_oracle.cpp")]
HDRS = [os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "csrc", "common", f) for f in ("rt_math.h", "rt_types.h")] + \
       [os.path.join(ROOT, "oracle", "glm_restated.h")]
LIB = os.path.join(ROOT, "tests", "_build", "libmath_pair.so")

OPS = {"add": 0, "sub": 1, "mul": 2, "scale": 3, "scale_left": 4, "div": 5, "neg": 6, "dot": 7, "cross": 8,
       "length": 9, "normalize": 10, "distance": 11, "clamp3": 12, "clamp": 13, "pow": 14, "mat4_point": 15,
       "mat3": 16, "max0": 17, "set_pixel": 18, "min1_max0": 19}


def _lib():
    deps = NATIVE + HDRS
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
                        "-o", LIB] + NATIVE, check=True)
    L = C.CDLL(LIB)
    for f in (L.math_pair_product, L.math_pair_oracle):
        f.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    return L


def _inputs(n, seed):
    """Vectors and matrices over many magnitudes, plus the edges: +-0,
    denormals, huge values (overflow in products), inf and NaN."""
    rng = np.random.default_rng(seed)

    def vecs():
        v = rng.normal(size=(n, 3))
        scale = 10.0 ** rng.uniform(-300, 300, size=(n, 1))
        v = v * np.where(rng.random((n, 1)) < 0.5, 1.0, scale)
        edge = np.array([0.0, -0.0, 5e-324, -5e-324, 2.2e-308, 1e-160, 1e160, 1.7e308, -1.7e308, np.inf, -np.inf,
                         np.nan, 1.0, -1.0, 0.5])
        pick = rng.random((n, 3)) < 0.1
        v[pick] = rng.choice(edge, size=pick.sum())
        return np.ascontiguousarray(v)

    a, b = vecs(), vecs()
    m = rng.normal(size=(n, 16)) * 10.0 ** rng.uniform(-3, 3, size=(n, 1))
    m[:, 3] = m[:, 7] = m[:, 11] = 0.0  # affine: last row (0, 0, 0, 1) (scene.h:64-135 matrices)
    m[:, 15] = 1.0
    pick = rng.random(m.shape) < 0.05
    m[pick] = rng.choice(np.array([0.0, -0.0, 1.0, -1.0, 1e-300, 1e300]), size=pick.sum())
    return a, b, np.ascontiguousarray(m)


def _same_bits(x, y):
    """Bit-identical, NaN payloads aside (both NaN counts as equal)."""
    xi, yi = x.view(np.uint64), y.view(np.uint64)
    return (xi == yi) | (np.isnan(x) & np.isnan(y))


@pytest.mark.parametrize("op", list(OPS))
def test_product_math_equals_oracle_glm(op):
    L = _lib()
    n = 50000
    for seed in (1, 2, 3):
        a, b, m = _inputs(n, seed)
        if op in ("pow",):
            a = np.abs(a)  # kt^t: kt >= 0 (material.cpp), t any
        if op in ("set_pixel",):
            a = np.clip(a, 0.0, 1.0)  # setPixel sees clamped colours (or NaN)
            a[::97] = np.nan
        outp = np.zeros_like(a)
        outo = np.zeros_like(a)
        assert L.math_pair_product(OPS[op], n, a.ctypes.data, b.ctypes.data, m.ctypes.data, outp.ctypes.data) == 0
        assert L.math_pair_oracle(OPS[op], n, a.ctypes.data, b.ctypes.data, m.ctypes.data, outo.ctypes.data) == 0
        ok = _same_bits(outp, outo)
        bad = np.nonzero(~ok.all(axis=1))[0]
        assert len(bad) == 0, (f"{op}: {len(bad)} of {n} results differ (seed {seed}); first a={a[bad[0]]} "
                               f"b={b[bad[0]]} product={outp[bad[0]]} oracle={outo[bad[0]]}")


def test_oracle_never_includes_product_math():
    """No oracle translation unit includes rt_math.h, directly or through the
    shared headers (scene_model.h, raw_records.h, image_io.cpp); the oracle's
    Makefile does not list it."""
    odir = os.path.join(ROOT, "oracle")
    srcs = [os.path.join(odir, f) for f in ("oracle.cpp", "parse_restated.cpp", "scene_build_restated.cpp",
                                            "ray_oracle_main.cpp")]
    srcs.append(os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "csrc", "host", "image_io.cpp"))
    for s in srcs:
        deps = subprocess.run(["g++", "-std=c++17", "-I" + os.path.join(ROOT, "include"), "-M", s], check=True,
                              capture_output=True, text=True).stdout
        assert "rt_math.h" not in deps, f"{os.path.basename(s)} includes rt_math.h"
    mk = open(os.path.join(odir, "Makefile")).read()
    assert "rt_math.h" not in mk.split("HDR      :=")[1].splitlines()[0]
