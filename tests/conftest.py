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
