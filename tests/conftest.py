"""Test configuration: puts the package root (convnet-quantization_amd/, so
``qconvnet``, ``models``, ``utils`` import the way the reference's modules do)
and the repo root (``oracle``) on sys.path, and registers the ``gpu`` marker."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "convnet-quantization_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
