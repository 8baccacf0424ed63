import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def built():
    """Native library, CLI and oracle, built in-tree (no-op when up to date)."""
    from fscl_amd import build
    build.build_native()
    build.build_oracle()
    return ROOT


@pytest.fixture
def tmp(tmp_path):
    return tmp_path
