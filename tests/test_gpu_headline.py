"""The headline configuration end to end on the GPU, so that pytest -m gpu
alone verifies what bench.py measures: the reference benchmark
(debian/extra/einstein_bench/bench_single.sh:28: the shipped 2^22-sample WU,
all 6662 templates of stochastic_full.bank, -A 0.08 -P 3.0 -f 400.0 -W)
against the CPU golden model's full-bank run (tools/make_golden.py), and the
reference's smoke target (debian/patches/benchmark.patch: the first 200
templates at -A 0.04 -P 3.0 -W -z) through the BOINC application binary."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import bench
from boinc_app_eah_brp_amd.models import BRPSearch, SearchConfig
from boinc_app_eah_brp_amd.models.search import app_binary

from conftest import BANK, ROOT, WU, ZAP

pytestmark = pytest.mark.gpu

GOLDEN = ROOT / "data" / "golden"


@pytest.fixture(scope="module")
def full_runs(tmp_path_factory):
    d = tmp_path_factory.mktemp("headline")
    os.environ["BRP_NO_RESULT_HEADER"] = "1"
    runs = {}
    for pipes in (1, 3):
        cfg = SearchConfig.benchmark(str(WU), str(BANK), str(ZAP), outputfile=str(d / f"p{pipes}.cand"), batch=1)
        runs[pipes] = BRPSearch(cfg, pipelines=pipes).run(use_checkpoint=False)
    return d, runs


def test_full_bench_wu_recall_vs_golden(brp, gpu, full_runs):
    """All 6662 templates: table recall 1.0 (240 golden entries) and
    result-line recall 1.0 (100 golden lines)."""
    _, runs = full_runs
    for pipes, r in runs.items():
        assert r.templates_run == 6662
        rec = bench.recall_vs_golden(r.table, r.geometry)
        assert rec is not None
        assert rec["golden_lines"] == 100 and rec["golden_entries"] == 240, rec
        assert rec["results"] == 1.0 and rec["table"] == 1.0, (pipes, rec)


def test_full_bench_wu_pipelines_byte_identical(brp, gpu, full_runs):
    """One and three pipelines per GPU: the same table and result file byte
    for byte (in-order application of the batches)."""
    d, runs = full_runs
    assert bytes(runs[1].table.to_bytes()) == bytes(runs[3].table.to_bytes())
    assert (d / "p1.cand").read_bytes() == (d / "p3.cand").read_bytes()


def test_full_bench_wu_powers_vs_golden(brp, gpu, full_runs):
    """Table powers of the common entries within float-FFT tolerance of the
    double-precision golden model."""
    _, runs = full_runs
    gt = brp.CandidateTable()
    gt.from_bytes(np.frombuffer((GOLDEN / "bench_wu_cpu_table.bin").read_bytes(), dtype=np.uint8).copy())
    gold = {(k // 100, int(e[0])): e[1] for k, e in enumerate(gt.entries()) if e[5] > 0}
    ours = {(k // 100, int(e[0])): e[1] for k, e in enumerate(runs[3].table.entries()) if e[5] > 0}
    rel = [abs(ours[k] - v) / v for k, v in gold.items()]
    assert max(rel) < 2e-4, max(rel)


def test_reference_smoke_200_templates(brp, gpu, tmp_path):
    """The reference's Debian test target through the application binary:
    first 200 templates, -A 0.04 -P 3.0 -W -z; result lines match the CPU
    golden model's 200-template run (tools/make_golden.py --end 200 --fA 0.04 --f0 250)."""
    golden = GOLDEN / "bench_wu_cpu_results_first200_A0.04_f250.txt"
    bank200 = tmp_path / "first200.bank"
    with open(BANK) as fh:
        bank200.write_text("".join(fh.readline() for _ in range(200)))
    args = [str(app_binary()), "-i", str(WU), "-t", str(bank200), "-l", str(ZAP), "-o", str(tmp_path / "res.cand"),
            "-c", str(tmp_path / "cp.cpt"), "-A", "0.04", "-P", "3.0", "-W", "-z"]
    env = dict(os.environ, BRP_NO_RESULT_HEADER="1")
    r = subprocess.run(args, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = r.stdout + r.stderr
    assert "thr16 = " in out  # -z: derived search parameters are logged
    lines, done = brp.read_results(str(tmp_path / "res.cand"))
    assert done and lines
    glines, gdone = brp.read_results(str(golden))
    assert gdone and len(glines) == len(lines)
    key = lambda ln: (round(ln[0], 6), ln[6])  # noqa: E731  (f0 [Hz], n_harm)
    assert {key(x) for x in lines} == {key(x) for x in glines}
    for a, b in zip(sorted(lines, key=key), sorted(glines, key=key)):
        assert a[4] == pytest.approx(b[4], rel=2e-4)
