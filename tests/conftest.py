import os

if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:  # libskm runs up to 12 streams (read at HIP init)
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def skm():
    import signature_kmers_amd as skm_mod
    if not os.path.exists(skm_mod.LIB_PATH):  # fresh checkout: build libskm.so + the oracle in-tree
        import subprocess
        subprocess.check_call(["make", "-C", ROOT, "-j", str(min(16, os.cpu_count() or 8)), "all"])
    skm_mod.lib()
    return skm_mod


@pytest.fixture(scope="session")
def gpu(skm):
    n = skm.device_count()
    if n < 1:
        pytest.fail("gpu test selected but no HIP device is visible")
    return 0
