"""The reference-side binding of INTEGRATION.md §2: include/rtx_traceui.h's
adapter (TraceUI flags -> RtxRenderParams) is compiled against the
UNMODIFIED /root/reference/ray/src/ui/TraceUI.h (tests/native/
traceui_adapter_check.cpp: explicit instantiation + accessor signature
asserts), and for every parity-case flag set it yields the RtxRenderParams
that RenderOptions.from_cli (the Python mirror the GPU tests use) yields.

Build container only (the reference is absent on the GPU box)."""
import os
import subprocess

import pytest

from cases import CASES
from conftest import ROOT

REF_UI = "/root/reference/ray/src/ui"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF_UI), reason="reference sources absent (GPU box)")

EXTRA_FLAGS = [
    "-w 1920 -r 5 -O r -A 4", "-w 1024 -r 5 -O r -A 4", "-w 1920 -r 5 -O d -A 2.5 -B 16 -C 0.05",
    "-w 3840 -r 5 -O a -A 8", "-w 64 -O j -A 3", "-w 32 -O c -A 0.25 -O s -A 7", "-O g -O o -r 2",
    "-O a -A 5 -B 0.125", "-O d -A 0.5 -B 0 -C 0.2",
]


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("adapter") / "traceui_adapter_check")
    subprocess.run(["g++", "-std=c++14", "-O1", "-Wall", "-Werror", f"-I{REF_UI}", f"-I{ROOT}/include", "-o", exe,
                    os.path.join(ROOT, "tests", "native", "traceui_adapter_check.cpp")], check=True)
    return exe


def test_adapter_matches_python_mirror(pkg, checker):
    flag_sets = sorted({c[2] for c in CASES} | set(EXTRA_FLAGS))
    lines = [f"{97 + k} {61 + k} {f}" for k, f in enumerate(flag_sets)]
    out = subprocess.run([checker], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    rows = out.stdout.strip().splitlines()
    assert len(rows) == len(flag_sets)
    names = ["width", "height", "depth", "aa_mode", "aa_samples", "dof", "dof_div", "anaglyph", "ss_res",
             "overlapping", "aa_thresh", "aterm_thresh", "dof_fd", "dof_apsz", "tile", "shard", "nshards", "packed"]
    for k, (flags, row) in enumerate(zip(flag_sets, rows)):
        assert row != "ERROR", flags
        vals = row.split()
        p = pkg.RenderOptions.from_cli(flags.split()).params(61 + k)
        for name, v in zip(names, vals):
            want = getattr(p, name)
            if name == "width":  # the C++ side was given the buffer width, as traceImage(w, h) is
                want = 97 + k
            got = float(v) if isinstance(want, float) else int(v)
            assert got == want, (flags, name, got, want)
