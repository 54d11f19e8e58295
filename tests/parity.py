"""The parity bar (BASELINE.json north_star), shared by the GPU tests and
bench.py's parity block: pixel RGB within 1e-4 absolute; object, face, scene
BVH leaf, mesh BVH leaf and per-sample ray counts bit-exact; primary hit t
bit-exact; 8-bit output identical except where the oracle's 255*c sits within
1e-9 of an integer (the truncation boundary of setPixel, RayTracer.cpp:388-394,
only reachable through a last-ulp difference of device pow)."""
import numpy as np

RGB_TOL = 1e-4
HIT_FIELDS = ("object", "face", "scene_leaf", "mesh_leaf", "nrays")


def measure(gpu_rgb, gpu_rgb8, ref_rgb, ref_rgb8, gpu_hits=None, ref_hits=None):
    """Mismatch figures of one frame (or band): max |rgb diff| (NaN must meet
    NaN: -O o media), rgb8 channels that differ off the truncation boundary,
    hit records whose fields differ, primary hits whose t differs."""
    assert gpu_rgb.shape == ref_rgb.shape, (gpu_rgb.shape, ref_rgb.shape)
    gn, rn = np.isnan(gpu_rgb), np.isnan(ref_rgb)
    nan_mismatch = int((gn != rn).sum())
    d = np.abs(np.where(rn, 0.0, gpu_rgb) - np.where(rn, 0.0, ref_rgb))
    scaled = 255.0 * ref_rgb
    boundary = np.abs(scaled - np.round(scaled)) < 1e-9
    bad8 = (gpu_rgb8.astype(np.int32) != ref_rgb8.astype(np.int32)) & ~boundary
    # (most boundary channels are exact 0 / 255 — black or saturated — and
    # equal anyway: rgb8_mismatch_any counts every differing channel)
    any8 = gpu_rgb8.astype(np.int32) != ref_rgb8.astype(np.int32)
    out = {"max_abs_rgb": float(d.max()) if d.size else 0.0, "nan_mismatch": nan_mismatch,
           "rgb8_mismatch": int(bad8.sum()), "rgb8_mismatch_any": int(any8.sum()),
           "rgb8_on_boundary": int(boundary.sum()),
           "channels": int(d.size)}
    if gpu_hits is not None and ref_hits is not None:
        assert gpu_hits.shape == ref_hits.shape, (gpu_hits.shape, ref_hits.shape)
        per = {}
        any_bad = np.zeros(gpu_hits.shape, bool)
        for f in HIT_FIELDS:
            m = gpu_hits[f] != ref_hits[f]
            per[f] = int(m.sum())
            any_bad |= m
        hit = ref_hits["object"] >= 0
        t_bad = int((gpu_hits["t"][hit] != ref_hits["t"][hit]).sum())
        out.update({"hit_mismatch": int(any_bad.sum()), "hit_field_mismatch": per, "t_mismatch": t_bad,
                    "samples": int(gpu_hits.size)})
    return out


def assert_parity(m):
    assert m["nan_mismatch"] == 0, f"NaN pattern differs in {m['nan_mismatch']} channels"
    assert m["max_abs_rgb"] <= RGB_TOL, f"max |rgb diff| {m['max_abs_rgb']}"
    assert m["rgb8_mismatch"] == 0, f"{m['rgb8_mismatch']} rgb8 mismatches off the truncation boundary"
    if "hit_mismatch" in m:
        for f, n in m["hit_field_mismatch"].items():
            assert n == 0, f"hit field {f}: {n} / {m['samples']} samples differ"
        assert m["t_mismatch"] == 0, f"primary hit t not bit-exact in {m['t_mismatch']} samples"
