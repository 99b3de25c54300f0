"""Shared pytest setup: import paths, the `gpu` marker, scene/oracle fixtures."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


REFERENCE = Path(os.environ.get("RT_REFERENCE_DIR", "/root/reference"))


def have_reference() -> bool:
    return (REFERENCE / "src" / "shaders" / "fragment_shader_ray_tracing.glsl").exists()


@pytest.fixture(scope="session")
def env_maps():
    from rtamd import configs as cf
    return cf.load_env()


@pytest.fixture(scope="session")
def gpu_renderer():
    from rtamd.renderer import Renderer
    r = Renderer(0)
    yield r
    r.close()


@pytest.fixture(scope="session")
def gpu_dev_renderer():
    """A context of lib/librtamd_dev.so (-DRT_DEV): the development settings the test sets in the
    environment (monkeypatch) reach the library; the release library ignores them."""
    from rtamd.renderer import Renderer, dev_lib_path
    r = Renderer(0, lib_path=dev_lib_path())
    yield r
    r.close()
