import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
DATA = ROOT / "data" / "testwu"
WU = DATA / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000_1099.bin4"
BANK = DATA / "stochastic_full.bank"
ZAP = DATA / "p2030.20151015.G187.41-00.88.N.b2s0g0.00000.zap"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def brp():
    import boinc_app_eah_brp_amd as pkg

    return pkg.native()


@pytest.fixture(scope="session")
def has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture()
def gpu(has_gpu):
    # GPU tests must run on the device: fail loudly instead of skipping
    assert has_gpu, "test marked gpu but no HIP device is visible"
    return True


@pytest.fixture()
def tmpdir_path(tmp_path):
    return tmp_path


@pytest.fixture(autouse=True)
def _device_fault_check(request):
    """After every GPU test: synchronise the device and fail THIS test if any
    of its work faulted (brp.device_check: hipDeviceSynchronize +
    hipGetLastError; in the checked build also the kernel, source line and
    address of an out-of-bounds access or guard-zone write). A device fault is
    then charged to the test that caused it, not to whichever later call
    happens to notice it (round-5 verdict)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import boinc_app_eah_brp_amd as pkg

    pkg.native().device_check()
