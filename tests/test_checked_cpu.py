"""CPU side of the device-side debug build (csrc/hip/checked.hpp) and of the
round-6 plan-override validation: no GPU needed."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def test_product_build_is_not_checked(brp):
    assert brp.checked_build() is False
    assert callable(brp.device_check)


def test_checked_module_selected_by_env():
    """BRP_CHECKED=1 makes the package load the checked build (_brp_checked),
    which reports itself as such; nothing touches the GPU at import."""
    from boinc_app_eah_brp_amd import _build

    if not _build.checked_extension_path().exists():
        pytest.skip("checked build not built here (python -m boinc_app_eah_brp_amd._build --checked)")
    env = dict(os.environ, BRP_CHECKED="1", BRP_NO_AUTOBUILD="1")
    code = ("import boinc_app_eah_brp_amd as p; m = p.native(); "
            "print(m.__name__.rsplit('.', 1)[-1], m.checked_build(), m.DD_HEADER_SIZE)")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[-3:] == ["_brp_checked", "True", "1168"]


@pytest.mark.parametrize("spec,accepted", [
    ("256x192x256", True),     # a supported factorisation covering 2 Mb - 1
    ("192x256x256", False),    # L2 > L1
    ("128x64x320", False),     # too short
    ("512x512x320", True),     # the longest compiled factorisation (L2 L3 = 163 840 <= 2^18)
    ("250x192x256", False),    # unsupported pass-1 length
    ("garbage", False),
])
def test_bs_plan_override_validated(brp, monkeypatch, spec, accepted):
    """BRP_BS_PLAN (A/B) applies only a factorisation the enumeration itself
    could pick (L2 <= L1, L2 L3 within the twiddle table, length < 2^31,
    compiled lengths, covering 2 Mb - 1); anything else is ignored and the cost
    model's plan is used."""
    Mb = 5_662_310  # -P 2.7 on 2^22 samples: N / 2
    monkeypatch.delenv("BRP_BS_PLAN", raising=False)
    default = brp.bluestein_plan(Mb)
    monkeypatch.setenv("BRP_BS_PLAN", spec)
    got = brp.bluestein_plan(Mb)
    if accepted:
        l1, l2, l3 = (int(x) for x in spec.split("x"))
        assert got == (l1 * l2 * l3, l1, l2, l3)
    else:
        assert got == default
    assert got[0] >= 2 * Mb - 1
