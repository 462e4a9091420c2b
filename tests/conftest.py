import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP module)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the native libraries once if they are missing (prebuilt .so files
    travel to the GPU box, so nothing is rebuilt there)."""
    from parmmg_amd import build

    for path, fn in ((build.SYNTH_SO, build.build_synth), (build.ORACLE_SO, build.build_oracle),
                     (build.HIP_SO, build.build_hip), (build.HOST_SO, build.build_host)):
        if not os.path.exists(path):
            fn()
    yield
