"""GPU parity: the HIP path (through the C ABI) against the CPU restatement.

Bar (BASELINE.json north_star): pixel RGB within 1e-4 absolute; kd-node
(scene/mesh BVH leaf), object, face indices and per-sample ray counts
bit-exact; 8-bit output identical except where the oracle's 255*c sits within
1e-9 of an integer (truncation boundary, only reachable through a last-ulp
difference of device pow)."""
import os

import numpy as np
import pytest

from cases import CASES
from conftest import cli_opts, scene_path

pytestmark = pytest.mark.gpu


def _compare(gpu, ref, spp):
    assert gpu["rgb"].shape == ref["rgb"].shape
    # -O o media can make a colour NaN (an empty object stack averages with
    # 1/0, RayTracer.cpp:128 + scene.cpp:234); NaN must meet NaN
    gn, rn = np.isnan(gpu["rgb"]), np.isnan(ref["rgb"])
    assert np.array_equal(gn, rn), f"NaN pattern differs in {(gn != rn).sum()} channels"
    d = np.abs(np.where(rn, 0.0, gpu["rgb"]) - np.where(rn, 0.0, ref["rgb"]))
    assert d.max() <= 1e-4, f"max |rgb diff| {d.max()}"
    g8, r8 = gpu["rgb8"].astype(int), ref["rgb8"].astype(int)
    scaled = 255.0 * ref["rgb"]
    boundary = np.abs(scaled - np.round(scaled)) < 1e-9
    bad = (g8 != r8) & ~boundary
    assert not bad.any(), f"{bad.sum()} rgb8 mismatches off the truncation boundary"
    gh, rh = gpu["hits"], ref["hits"]
    for f in ("object", "face", "scene_leaf", "mesh_leaf", "nrays"):
        mism = (gh[f] != rh[f])
        assert not mism.any(), f"hit field {f}: {mism.sum()} / {mism.size} samples differ"
    hit = rh["object"] >= 0
    assert np.array_equal(gh["t"][hit], rh["t"][hit]), "primary hit t not bit-exact"


# render paths (DESIGN.md "Kernels"): the wavefront advance/trace pipeline
# (default, 3 slot groups on 3 streams), the persistent megakernel, one slot
# group, a tiny slot pool so every slot walks many samples (claim_sample's
# static deal), and the tail kernel finishing almost everything.  The small
# parity frames have fewer samples than slots, so "wavefront" forks ray
# sub-trees onto spare slots (heap depth 3); "wavefront_nofork" does not,
# "wavefront_fork4" forks down to depth 4
PATHS = {"wavefront": {}, "mega": {"RTX_MEGAKERNEL": "1"}, "wavefront_1g": {"RTX_GROUPS": "1"},
         "wavefront_256": {"RTX_SLOTS": "256"},
         "wavefront_nofork": {"RTX_FORK": "0"}, "wavefront_fork4": {"RTX_FORK_DEPTH": "4"},
         # tail_kernel takes over right after the first batched iteration
         "wavefront_tail": {"RTX_TAIL": "1000000000"}}


@pytest.fixture(params=list(PATHS), ids=list(PATHS))
def render_path(request):
    saved = {k: os.environ.get(k) for k in ("RTX_MEGAKERNEL", "RTX_SLOTS", "RTX_GROUPS", "RTX_TAIL", "RTX_FORK",
                                     "RTX_FORK_DEPTH")}
    for k in saved:
        os.environ.pop(k, None)
    os.environ.update(PATHS[request.param])
    yield request.param
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("name,scene,flags", CASES, ids=[c[0] for c in CASES])
def test_parity(pkg, orc, render_path, name, scene, flags):
    path = scene_path(scene)
    opts = cli_opts(pkg, flags)
    host = pkg.HostScene(path, cubemap=opts.cubemap)
    assert host.cubemap_error is None
    dev = pkg.DeviceScene(host, 0)
    gpu = dev.render(opts, want_f64=True, want_hits=True, stats=True)
    ref = orc.render(pkg, path, opts, want_hits=True)
    if opts.aa_mode == pkg.RTX_AA_ADAPTIVE:
        # only the top-level region's samples carry records
        pass
    _compare(gpu, ref, opts.spp)
    # whole-frame ray counts (camera + secondary + shadow) agree
    for k in ("camera_rays", "secondary_rays", "shadow_rays"):
        assert gpu["stats"][k] == ref["stats"][k], (k, gpu["stats"][k], ref["stats"][k])


def test_sharded_tiles_reassemble(pkg, render_path):
    """Tile sharding: packed shards reassemble to the full frame."""
    path = scene_path("hitchcock.ray")
    opts = pkg.RenderOptions.from_cli("-w 100 -r 2 -O r -A 2".split())
    host = pkg.HostScene(path)
    dev = pkg.DeviceScene(host, 0)
    full = dev.render(opts, want_f64=True)
    h = full["height"]
    out8 = np.zeros((h, opts.width, 3), np.uint8)
    outf = np.zeros((h, opts.width, 3), np.float64)
    for shard in range(3):
        part = dev.render(opts, want_f64=True, tile=32, shard=shard, nshards=3, packed=True)
        pkg.unpack_tiles(part["rgb8"], opts.width, h, 32, shard, 3, out8)
        pkg.unpack_tiles(part["rgb"], opts.width, h, 32, shard, 3, outf)
    assert np.array_equal(out8, full["rgb8"])
    assert np.array_equal(outf, full["rgb"])


def test_repeat_deterministic(pkg):
    path = scene_path("spheres_overlap.ray")
    opts = pkg.RenderOptions.from_cli("-w 64 -r 5 -O r -A 2".split())
    dev = pkg.DeviceScene(pkg.HostScene(path), 0)
    a = dev.render(opts)
    b = dev.render(opts)
    assert np.array_equal(a["rgb"], b["rgb"])


def test_no_device_fallback_error(pkg):
    """Bad device index fails loudly (no CPU fallback)."""
    host = pkg.HostScene(scene_path("spheres_overlap.ray"))
    with pytest.raises(pkg.RtxError):
        pkg.DeviceScene(host, 97)
