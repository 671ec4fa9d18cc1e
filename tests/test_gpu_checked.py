"""Device-side debug mode (csrc/hip/checked.hpp): the checked
build (module _brp_checked) runs the benchmark geometry's whitened batch with
bounds-checked kernel accesses, verified launches and guard zones, and
reports an injected out-of-bounds access with the kernel's name. Each case
runs in a child process (the checked module and the injection are chosen at
start-up)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
RUN = Path(__file__).resolve().parent / "_checked_run.py"


def _run(*args, inject=None, timeout=240):
    env = dict(os.environ)
    env.pop("BRP_CHECKED_INJECT", None)
    if inject:
        env["BRP_CHECKED_INJECT"] = inject
    r = subprocess.run([sys.executable, "-u", str(RUN), *args], capture_output=True, text=True, timeout=timeout,
                       env=env, cwd=str(ROOT))
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line), r.stderr


def test_checked_bench_batch_clean(gpu):
    """The whitened 2-template batch of the benchmark geometry (whitening
    kernels, pass 1 / 2 / 3, hs_cells, hs_pruned), then the test hooks
    (bound_cells, power_spectrum, download_series): every launch verified,
    every instrumented access inside its allocation, no guard zone touched,
    every host copy from pinned memory; the cells equal the spectrum's 8-bin
    maxima as in the product build."""
    out, err = _run("--hooks")
    assert out["checked"] is True
    assert out["process_error"] is None, err[-3000:]
    assert out["hooks_error"] is None, err[-3000:]
    assert out["device_check"] == "clean", err[-3000:]
    assert out["cells_ok"] is True
    assert "checked:" not in err, err[-3000:]


@pytest.mark.parametrize("site,kernel,kind", [("hs_cells", "hs_cells_kernel", "store"),
                                              ("pass1", "pass1_pruned3_kernel", "load"),
                                              ("pass3", "pass3_kernel", "store"),
                                              ("hs_pruned", "hs_pruned_kernel", "load")])
def test_checked_reports_injected_oob(gpu, site, kernel, kind):
    """An out-of-bounds index injected into one thread (test-only,
    BRP_CHECKED_INJECT) is caught before the access, the launch fails, and the
    report names the kernel, the access and the address just past the
    allocation; the device check after it carries the same report."""
    out, err = _run(inject=site)
    assert out["process_error"] is not None, (out, err[-3000:])
    assert f"checked: kernel ({kernel}" in err, err[-3000:]
    assert f"out-of-bounds {kind}" in err and "past its end" in err, err[-3000:]
    assert kernel in out["device_check"], out
