"""tools/raycheck.py — the counterpart of the reference's grading harness
(ray/raycheck.py): image readers, RMS with and without the uint8 wrap, and an
end-to-end run (CPU: the restatement against itself; GPU: bin/ray against the
restatement under the strict north-star bar)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import NEWSCENE, ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import raycheck  # noqa: E402

ORACLE_BIN = os.path.join(ROOT, "oracle", "_build", "ray_oracle")
RAY_BIN = os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "bin", "ray")


def _oracle_bin(orc):
    if not os.path.exists(ORACLE_BIN):
        orc.build()
    return ORACLE_BIN


def test_rms_wrap():
    a = np.array([0, 10, 255], np.uint8)
    b = np.array([1, 10, 0], np.uint8)
    wrapped, true = raycheck.rms(a, b)
    # 0-1 wraps to 255 in uint8 (the reference's behaviour)
    assert wrapped == pytest.approx(np.sqrt((255.0 ** 2 + 255.0 ** 2) / 3))
    assert true == pytest.approx(np.sqrt((1.0 + 255.0 ** 2) / 3))


def test_png_reader_matches_dump(orc, tmp_path):
    """PNG written by the CLI decodes to the truncated f64 image, top row first."""
    exe = _oracle_bin(orc)
    png = str(tmp_path / "o.png")
    f64 = str(tmp_path / "o.f64")
    rc = subprocess.run([exe, "-w", "24", "-r", "2", "--dump-f64", f64,
                         os.path.join(NEWSCENE, "spheres_overlap.ray"), png]).returncode
    assert rc == 0
    img = raycheck.read_png(png)
    raw = np.fromfile(f64, np.float64)
    h = raw.size // (24 * 3)
    buf = (255.0 * raw).astype(np.int64).astype(np.uint8).reshape(h, 24, 3)  # row 0 = bottom
    assert np.array_equal(img, buf[::-1])


def test_bmp_reader():
    img = raycheck.read_bmp(os.path.join(NEWSCENE, "lava_texture.bmp"))
    assert img.ndim == 3 and img.shape[2] == 3 and img.dtype == np.uint8
    assert img.size > 0


def test_self_check_passes(orc, tmp_path):
    exe = _oracle_bin(orc)
    rc = raycheck.main(["--exec", exe, "--ref", exe, "--scenes", NEWSCENE, "--out", str(tmp_path / "rc"),
                        "--flags", "-w 16", "--strict"])
    assert rc == 0


@pytest.mark.gpu
def test_raycheck_gpu_vs_restatement(orc, tmp_path):
    """bin/ray (HIP path) against the CPU restatement on every bundled scene,
    the harness's own RMS bar plus the strict bar (1e-4, ids bit-exact)."""
    exe = _oracle_bin(orc)
    rc = raycheck.main(["--exec", RAY_BIN, "--ref", exe, "--scenes", NEWSCENE, "--out", str(tmp_path / "rc"),
                        "--flags", "-w 48", "--strict"])
    assert rc == 0
