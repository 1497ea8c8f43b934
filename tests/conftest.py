import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built():
    lib = os.path.join(ROOT, "m2dec_amd", "lib", "libm2dec_amd.so")
    orc = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc)):
        subprocess.run(["make", "-C", ROOT, "-j8"], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def built():
    _ensure_built()
    return ROOT
