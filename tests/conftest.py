import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
SCENE = os.path.join(GOLDEN, "example", "scene.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def scene_path():
    return SCENE


@pytest.fixture(scope="session")
def py_scene():
    from oracle.scene_py import load_scene
    return load_scene(SCENE)


@pytest.fixture(scope="session")
def oracle(py_scene):
    from oracle.oracle import Oracle
    return Oracle(py_scene)


@pytest.fixture(scope="session")
def ctx():
    import distributed_raytracer_amd as rt
    return rt.Context(0)


@pytest.fixture(scope="session")
def env(ctx):
    import distributed_raytracer_amd as rt
    return rt.Environment.from_file(SCENE, ctx)
