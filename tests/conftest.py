import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs the HIP path")


@pytest.fixture(scope="session")
def ctx():
    """One pitt context on cuda:0 for the whole GPU session (tests share it, run in one process)."""
    import torch  # noqa: F401  (loads the HIP runtime the library binds to)
    from pitt_object_table_segmentation_amd import Context
    c = Context(0)
    yield c
    c.close()
