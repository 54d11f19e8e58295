"""Shared fixtures.  `gpu` marks tests that need a real MI355X (gfx950)."""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
NEWSCENE = os.path.join(GOLDEN, "newScene")
FEATURE = os.path.join(GOLDEN, "feature")
SCENES = os.path.join(ROOT, "scenes")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu)")


def load_package():
    name = "cs378hgraphics_raytracer_amd"
    if name in sys.modules:
        return sys.modules[name]
    path = os.path.join(ROOT, "cs378hgraphics-raytracer_amd", "__init__.py")
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (test infrastructure)
    return oracle


@pytest.fixture(scope="session")
def pkg():
    return load_package()


@pytest.fixture(scope="session")
def orc():
    o = load_oracle()
    if not os.path.exists(o.LIB):
        o.build()
    return o


def cli_opts(pkg, flags):
    """RenderOptions from reference CLI flags; a relative -c path names a
    cube-map face under tests/golden (e.g. cubemap/posx.bmp)."""
    opts = pkg.RenderOptions.from_cli(flags.split())
    if opts.cubemap and not os.path.isabs(opts.cubemap):
        opts.cubemap = os.path.join(GOLDEN, opts.cubemap)
    return opts


def scene_path(name):
    for d in (NEWSCENE, FEATURE, SCENES, GOLDEN, os.path.join(GOLDEN, "kat")):
        p = os.path.join(d, name)
        if os.path.exists(p):
            return p
    raise FileNotFoundError(name)
