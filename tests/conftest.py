import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels through the C-ABI)")


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (tests/ may use it as the checker; never the product)."""
    from tests import oracle_lib

    return oracle_lib.load()
