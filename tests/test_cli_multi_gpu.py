"""`bin/ray --gpus N` — the product's multi-GPU driver (csrc/host/multi_gpu.cpp):
one process per GPU, 32x32 tiles dealt over the ranks, packed RGB8 shards
gathered to rank 0 over RCCL (ncclGather), reassembled with rtx_unpack_tiles.
The image must equal the single-GPU render of the same command bit for bit
(the sharded kernels accumulate in the same order: DESIGN.md §5).

The reassembly half (rtx_shard_tiles / rtx_unpack_tiles, the code the
driver's rank 0 runs) is checked on CPU over a world-size-2 gloo gather in
test_distributed_gloo.py."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, scene_path

RAY_BIN = os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "bin", "ray")


def _run(args, timeout=240):
    return subprocess.run([RAY_BIN] + args, capture_output=True, text=True, timeout=timeout)


def test_gpus_argument_checked():
    """Refused before any process is forked or any device is touched."""
    r = _run(["--gpus", "65", scene_path("hitchcock.ray"), "/tmp/never.png"])
    assert r.returncode == 1 and "--gpus" in r.stderr
    r = _run(["--gpus", "2", "--dump-f64", "/tmp/x.f64", scene_path("hitchcock.ray"), "/tmp/never.png"])
    assert r.returncode == 1 and "single-GPU" in r.stderr


def _device_count(pkg):
    import ctypes as C

    n = C.c_int()
    pkg.hip_lib().rtx_device_count(C.byref(n))
    return n.value


@pytest.mark.gpu
@pytest.mark.parametrize("scene,flags", [
    ("trimesh2_square.ray", "-w 96 -r 5 -O r -A 2"),
    ("hitchcock.ray", "-w 80 -r 3"),
])
def test_multi_gpu_cli_equals_single(pkg, tmp_path, scene, flags):
    path = scene_path(scene)
    single = tmp_path / "single.png"
    r = _run(flags.split() + [path, str(single)])
    assert r.returncode == 0, r.stderr
    want = pkg.read_image(str(single))
    counts = [1] + ([2] if _device_count(pkg) >= 2 else [])
    for n in counts:
        out = tmp_path / f"gpus{n}.png"
        r = _run(["--gpus", str(n), "--stats"] + flags.split() + [path, str(out)])
        assert r.returncode == 0, r.stderr
        got = pkg.read_image(str(out))
        assert np.array_equal(got, want), f"--gpus {n} differs from the single-GPU render"
        assert '"gpus": %d' % n in r.stdout


def test_bad_numeric_options_refused():
    """--gpus / --tile / --device take whole numbers in range:
    no silent fallback to one GPU or to the default tiles."""
    for args in (["--gpus", "abc"], ["--gpus", "0"], ["--tile", "0"], ["--tile", "-4"], ["--device", "x1"]):
        r = _run(args + [scene_path("hitchcock.ray"), "/tmp/never.png"])
        assert r.returncode == 1, (args, r.returncode, r.stderr)
        assert "--" + args[0].lstrip("-") in r.stderr


@pytest.mark.gpu
def test_multi_gpu_more_ranks_than_devices_fails_fast(pkg, tmp_path):
    """A rank that cannot come up (here: more ranks than visible GPUs) makes
    the job exit non-zero within a bound instead of leaving the other ranks
    blocked in ncclCommInitRank / ncclGather (multi_gpu.cpp: the rendezvous
    page's failure flag and the parent's termination of the remaining
    ranks)."""
    import time

    n = _device_count(pkg) + 1
    t0 = time.monotonic()
    r = _run(["--gpus", str(n), "-w", "32", scene_path("hitchcock.ray"), str(tmp_path / "x.png")], timeout=90)
    assert r.returncode != 0, r.stdout
    assert time.monotonic() - t0 < 60
    assert "no GPU" in r.stderr, r.stderr
