import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
if os.path.join(ROOT, "tests") not in sys.path:
    sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP datapath)")


@pytest.fixture(scope="session", autouse=True)
def _built_libs():
    """Build the oracle (and the product .so if missing) once per session."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "polycube_amd", "libpcn_ipt.so")):
        subprocess.run(["make", "-s", "-j4", "-C", os.path.join(ROOT, "polycube_amd")], check=True)
