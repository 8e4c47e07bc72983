import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def build_host_tool(target):
    """make a scripts/ host harness under an exclusive lock: parallel test workers must not
    run a binary another worker is relinking."""
    import fcntl

    os.makedirs(os.path.join(ROOT, "scripts", "build"), exist_ok=True)
    with open(os.path.join(ROOT, "scripts", "build", ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.check_call(["make", "-s", "-j4", "-C", os.path.join(ROOT, "scripts"), target])
    return os.path.join(ROOT, "scripts", "build", target)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels through the C-ABI)")


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (tests/ may use it as the checker; never the product)."""
    from tests import oracle_lib

    return oracle_lib.load()
